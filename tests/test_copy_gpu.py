"""Device -> host copies as GPU stores into pinned host memory
(copy_kernels.hip, rt_memcpy_d2h, device.copy_to_host): every byte arrives,
at any size and alignment, pinned or pageable destination, and the bytes
around a destination view are left alone."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


SIZES = [1, 2, 15, 16, 17, 31, 33, 255, 4096 + 3, (1 << 20) + 7, (64 << 20) + 13]


@pytest.mark.parametrize("pinned", [True, False])
@pytest.mark.parametrize("size", SIZES)
@pytest.mark.parametrize("dst_off,src_off", [(0, 0), (3, 0), (0, 5), (9, 9), (15, 1)])
def test_copy_to_host_exact(dev, pinned, size, dst_off, src_off):
    from reticulum_amd import device
    if size > (1 << 21) and (dst_off, src_off) not in ((0, 0), (3, 0)):
        pytest.skip("large sizes at two alignments only")
    g = torch.Generator(device=dev).manual_seed(size * 31 + dst_off * 7 + src_off)
    src_buf = torch.randint(0, 256, (size + 32,), dtype=torch.uint8, device=dev, generator=g)
    host = torch.full((size + 32,), 0xEE, dtype=torch.uint8)
    if pinned:
        host = host.pin_memory()
    src = src_buf[src_off:src_off + size]
    dst = host[dst_off:dst_off + size]
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    device.copy_to_host(dst, src, stream=s)
    s.synchronize()
    assert torch.equal(dst, src.cpu())
    # the bytes before and after the view are untouched
    assert bool((host[:dst_off] == 0xEE).all()) and bool((host[dst_off + size:] == 0xEE).all())


def test_copy_to_host_rejects_bad_args(dev):
    from reticulum_amd import device
    d = torch.zeros(16, dtype=torch.uint8, device=dev)
    with pytest.raises(ValueError):
        device.copy_to_host(torch.zeros(15, dtype=torch.uint8), d)
    with pytest.raises(ValueError):
        device.copy_to_host(d, d)
    with pytest.raises(ValueError):
        device.copy_to_host(torch.zeros(32, dtype=torch.uint8)[::2], d)


def test_copy_to_host_ordered_after_kernel_on_stream(dev):
    """The stores run after the work enqueued before them on the same stream:
    100 rounds of fill -> copy on one side stream, each checked."""
    from reticulum_amd import device
    s = torch.cuda.Stream(device=dev)
    src = torch.empty(3 << 20, dtype=torch.uint8, device=dev)
    dst = torch.empty(3 << 20, dtype=torch.uint8).pin_memory()
    with torch.cuda.stream(s):
        for r in range(100):
            src.fill_(r)
            device.copy_to_host(dst, src, stream=s)
            s.synchronize()
            assert int(dst[0]) == r and int(dst[-1]) == r and bool((dst == r).all())


@pytest.mark.parametrize("dst_off", [0, 3, 13])
def test_copy_to_host_upto_clamps_on_the_device(dev, dst_off):
    """rt_memcpy_d2h_upto: the count is read on the device and clamped to
    [0, max]: 0, 1..15 (inside the unaligned head), a middle count, more than
    the destination holds, and a negative int64 (nothing copied); bytes past
    the count are untouched."""
    from reticulum_amd import device
    size = 4096 + 37
    g = torch.Generator(device=dev).manual_seed(77 + dst_off)
    src = torch.randint(0, 256, (size,), dtype=torch.uint8, device=dev, generator=g)
    ref = src.cpu()
    for want in [0, 1, 2, 7, 15, 16, 17, 1000, size - 1, size, size + 100, 1 << 40, -1, -4096]:
        host = torch.full((size + 32,), 0xEE, dtype=torch.uint8).pin_memory()
        dst = host[dst_off:dst_off + size]
        nb = torch.tensor([want], dtype=torch.int64, device=dev)
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        device.copy_to_host_upto(dst, src, nb, stream=s)
        s.synchronize()
        k = max(0, min(want, size))
        assert torch.equal(dst[:k], ref[:k]), want
        assert bool((dst[k:] == 0xEE).all()), want
        assert bool((host[:dst_off] == 0xEE).all()) and bool((host[dst_off + size:] == 0xEE).all()), want


def test_copy_to_host_upto_rejects_bad_counts(dev):
    from reticulum_amd import device
    src = torch.zeros(64, dtype=torch.uint8, device=dev)
    dst = torch.zeros(64, dtype=torch.uint8).pin_memory()
    with pytest.raises(TypeError):
        device.copy_to_host_upto(dst, src, torch.tensor([3], dtype=torch.int32, device=dev))
    with pytest.raises(TypeError):
        device.copy_to_host_upto(dst, src, torch.tensor([3], dtype=torch.int64))        # on the host
    with pytest.raises(TypeError):
        device.copy_to_host_upto(dst, src, torch.tensor([3, 4], dtype=torch.int64, device=dev))
