"""In-run launch clock (rt_clock_stamps, device.LaunchClock): every stamped
launch adds one span per workgroup; the spans agree with the HIP-event time
of the launches; the sustained clock is a plausible MI355X shader clock; the
stamps change no output byte and stop when the block ends."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _batch(n=1 << 18, L=500):
    import reticulum_amd as rt
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(5)
    pt = torch.randint(0, 256, (n, L), dtype=torch.uint8, device=dev, generator=g)
    iv = torch.randint(0, 256, (n, 16), dtype=torch.uint8, device=dev, generator=g)
    ks = rt.KeySet(bytes(range(64)), device=0)
    tl = rt.token_len(L)
    tok = torch.empty((n, tl), dtype=torch.uint8, device=dev)
    back = torch.empty((n, tl - 48), dtype=torch.uint8, device=dev)
    ol = torch.empty(n, dtype=torch.int32, device=dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    return dev, ks, pt, iv, tok, back, ol, st, L, tl


def test_launch_clock_spans_agree_with_events():
    from reticulum_amd import device, _native
    dev, ks, pt, iv, tok, back, ol, st, L, tl = _batch(1 << 20)
    s = torch.cuda.current_stream()
    for _ in range(10):          # clock ramp
        device.encrypt_uniform(ks, pt, L, iv, tok)
        device.decrypt_uniform(ks, tok, tl, back, ol, st)
    reps = 12
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(reps)]
    with device.LaunchClock(dev) as lc:
        for e in ev:
            e[0].record(s)
            device.encrypt_uniform(ks, pt, L, iv, tok)
            e[1].record(s)
            device.decrypt_uniform(ks, tok, tl, back, ol, st)
            e[2].record(s)
    summ = lc.summary()
    assert bool((st == 0).all()) and torch.equal(back[:, :L], pt)
    n_cu = _native.load().rt_num_cus(_native.context(0))
    for name, k in (("encrypt", 0), ("decrypt", 1)):
        r = summ[name]
        assert r["launches"] == reps, r
        assert 1 <= r["workgroups_per_launch"] <= n_cu, r          # one persistent workgroup per CU at most
        assert 0.8 < r["clock_ghz"] < 2.6, r
        ev_ms = sum(e[k].elapsed_time(e[k + 1]) for e in ev) / reps
        # a workgroup's span sits inside its launch and covers nearly all of it
        assert 0.75 * ev_ms < r["wg_span_ms"] <= 1.02 * ev_ms, (r, ev_ms)
        # cycles per launch = clock x span
        assert r["cycles_per_launch"] == pytest.approx(r["clock_ghz"] * 1e6 * r["wg_span_ms"], rel=1e-6)
    # stamping stopped with the block
    before = lc.words()
    device.encrypt_uniform(ks, pt, L, iv, tok)
    assert lc.words() == before


def test_launch_clock_changes_no_output():
    from reticulum_amd import device
    dev, ks, pt, iv, tok, back, ol, st, L, tl = _batch(1 << 16, 1500)
    device.encrypt_uniform(ks, pt, L, iv, tok)
    ref = tok.clone()
    with device.LaunchClock(dev) as lc:
        device.encrypt_uniform(ks, pt, L, iv, tok)
        device.decrypt_uniform(ks, tok, tl, back, ol, st)
    assert torch.equal(tok, ref) and bool((st == 0).all()) and torch.equal(back[:, :L], pt)
    assert lc.summary()["decrypt"]["launches"] == 1


def test_clock_stamps_rejects_host_memory():
    from reticulum_amd import _native
    import ctypes
    lib = _native.load()
    buf = (ctypes.c_uint64 * 8)()
    assert lib.rt_clock_stamps(_native.context(0), ctypes.addressof(buf)) < 0
    assert lib.rt_clock_stamps(_native.context(0), None) == 0


def test_launch_clock_stamps_long_token_kernels():
    """Batches of few packets per CU route to the long-token kernels
    (k_encrypt_long4 / k_decrypt_long2 for one key, k_encrypt_long per key):
    they stamp their launches too."""
    import reticulum_amd as rt
    from reticulum_amd import device, _native
    dev, ks, pt, iv, tok, back, ol, st, L, tl = _batch(1024, 500)
    lib, ctx = _native.load(), _native.context(0)
    assert lib.rt_plan_uniform(ctx, 1024, L, 0, 0) == _native.RT_KERNEL_ENC_LONG4
    assert lib.rt_plan_uniform(ctx, 1024, tl, 0, 1) == _native.RT_KERNEL_DEC_LONG2
    with device.LaunchClock(dev) as lc:
        device.encrypt_uniform(ks, pt, L, iv, tok)
        device.decrypt_uniform(ks, tok, tl, back, ol, st)
        kk = rt.KeySet([bytes(range(64)), bytes(range(64, 128))], device=0)     # two keys: the per-key long kernel
        kidx = (torch.arange(1024, device=dev, dtype=torch.int32) & 1).contiguous()
        device.encrypt_uniform(kk, pt, L, iv, tok, key_idx=kidx)
    s = lc.summary()
    assert bool((st == 0).all()) and torch.equal(back[:, :L], pt)
    assert s["encrypt"]["launches"] == 2 and s["decrypt"]["launches"] == 1, s
    assert 0.5 < s["encrypt"]["clock_ghz"] < 2.6 and 0.5 < s["decrypt"]["clock_ghz"] < 2.6, s
