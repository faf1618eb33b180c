"""device.aligned_rows: the row views the slot recommendation
hands to the uniform entry points — stride a multiple of 128, byte `phase` of
every row on a 128-B line, rows disjoint, whatever the allocation's own
alignment."""
import pytest


@pytest.mark.parametrize("n,width,phase", [(5, 500, 0), (7, 560, 16), (3, 451, 35), (1, 128, 0), (4, 129, 127),
                                           (2, 0, 0), (0, 10, 0), (1000, 1552, 16)])
def test_aligned_rows_geometry(n, width, phase):
    import torch
    from reticulum_amd import device
    r = device.aligned_rows(n, width, phase)
    assert tuple(r.shape) == (n, width) and r.dtype == torch.uint8
    if n:
        assert r.stride(1) == 1 and r.stride(0) % 128 == 0 and r.stride(0) >= max(width, 1)
        assert (r.data_ptr() + phase) % 128 == 0
        r.fill_(0)
        r[-1].fill_(1)                                  # the last row fits its buffer
        assert int(r[:-1].sum()) == 0                   # rows are disjoint


def test_aligned_rows_bad_args():
    from reticulum_amd import device
    for args in ((-1, 4, 0), (1, -4, 0), (1, 4, 128), (1, 4, -1)):
        with pytest.raises(ValueError):
            device.aligned_rows(*args)
