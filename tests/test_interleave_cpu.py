"""Host side of the unit-interleaved layout (reticulum_amd.device): the
layout helpers and the argument checks that run before any library call."""
import pytest
import torch

from reticulum_amd import device


@pytest.mark.parametrize("n,L", [(1, 0), (1, 1), (7, 15), (7, 16), (5, 17), (33, 500), (3, 4096)])
def test_interleave_layout(n, L):
    rows = torch.randint(0, 256, (n, max(L, 1)), dtype=torch.uint8)[:, :L]
    u = device.interleave(rows, L)
    U = (L + 15) // 16
    assert tuple(u.shape) == (U, n, 16) and u.is_contiguous()
    flat = u.reshape(-1)
    for p in range(n):
        for k in range(L):          # byte k of packet p sits at 16*((k//16)*n + p) + k%16
            assert int(flat[16 * ((k // 16) * n + p) + k % 16]) == int(rows[p, k])
    if L % 16:
        assert int(u[U - 1, :, L % 16:].abs().sum()) == 0          # padded tail unit
    assert torch.equal(device.deinterleave(u, L), rows.contiguous())


def test_interleaved_entry_checks_shapes_before_the_library():
    class KS:                       # never reached: the checks raise first
        handle = None
    n, L = 4, 40
    pt = torch.zeros((3, n, 16), dtype=torch.uint8)
    iv = torch.zeros((n, 16), dtype=torch.uint8)
    tok = torch.zeros((device.units(16 + 48 + 32), n, 16), dtype=torch.uint8)
    with pytest.raises(ValueError):          # wrong unit count
        device.encrypt_interleaved(KS, torch.zeros((2, n, 16), dtype=torch.uint8), L, iv, tok)
    with pytest.raises(ValueError):          # token buffer of the wrong length
        device.encrypt_interleaved(KS, pt, L, iv, torch.zeros((5, n, 16), dtype=torch.uint8))
    with pytest.raises(ValueError):          # host tensors: the device API refuses them
        device.encrypt_interleaved(KS, pt, L, iv, tok)
    ol = torch.zeros(n, dtype=torch.int32)
    with pytest.raises(ValueError):          # malformed token length
        device.decrypt_interleaved(KS, torch.zeros((4, n, 16), dtype=torch.uint8), 60, pt, ol, ol)
    with pytest.raises(ValueError):          # plaintext units for a different length
        device.decrypt_interleaved(KS, tok, 96, torch.zeros((2, n, 16), dtype=torch.uint8), ol, ol)
