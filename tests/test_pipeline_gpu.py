"""The interface path composed on the device (reticulum_amd.pipeline):
outbound token encrypt -> header pack -> IFAC mask -> HDLC framing gives
exactly the stream the reference's steps give (the oracle's restatements of
Token.encrypt, Packet.pack, Transport.transmit and HDLC.escape, each pinned to
reference-generated vectors), and inbound deframing -> IFAC unmask -> unpack
-> token decrypt of that stream gives back every packet, its IFAC, header
fields and plaintext; a tampered tag fails that packet alone."""
import numpy as np
import pytest

from oracle import ctoken
from oracle import wire as ow

pytestmark = pytest.mark.gpu


def _case(n, L, isz, seed):
    import torch
    rng = np.random.Generator(np.random.PCG64(seed))
    key = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
    ifac_key = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
    pt = rng.integers(0, 256, (n, L), dtype=np.uint8)
    iv = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    dh = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    ctx = rng.integers(0, 256, n, dtype=np.uint8)
    ifac = rng.integers(0, 256, (n, isz), dtype=np.uint8)
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    return key, ifac_key, pt, iv, dh, ctx, ifac, t


def _reference_stream(key, ifac_key, pt, iv, dh, ctx, ifac):
    frames = []
    for i in range(pt.shape[0]):
        tok = ctoken.encrypt(key, iv[i].tobytes(), pt[i].tobytes())
        raw = ow.pack_header(0, 0, dh[i].tobytes(), int(ctx[i])) + tok
        frames.append(ow.hdlc_frame(ow.ifac_mask(raw, ifac[i].tobytes(), ifac_key)))
    return b"".join(frames)


@pytest.mark.parametrize("n,L,isz", [(1500, 383, 16), (700, 17, 8), (257, 0, 16)])
def test_outbound_stream_is_the_references_and_inbound_returns_every_packet(n, L, isz):
    import torch
    import reticulum_amd as rt
    from reticulum_amd import pipeline
    key, ifac_key, pt, iv, dh, ctx, ifac, t = _case(n, L, isz, 100 + n + L)
    ks = rt.KeySet(key, device=0)
    framed, foff = pipeline.outbound(ks, t(pt), t(iv), t(dh), t(ctx), t(ifac), t(np.frombuffer(ifac_key, np.uint8)))
    total = int(foff[-1])
    stream = framed[:total].cpu().numpy().tobytes()
    assert stream == _reference_stream(key, ifac_key, pt, iv, dh, ctx, ifac)

    res = pipeline.inbound(ks, framed[:total].clone(), t(np.frombuffer(ifac_key, np.uint8)), isz, 2 * n)
    torch.cuda.synchronize()
    assert int(res["n_frames"]) == n and int(res["counts"][0]) == 2 * n - 1
    assert res["frame_pair"][:n].cpu().tolist() == list(range(0, 2 * n, 2))
    assert bool((res["ifac_status"][:n] == 0).all()) and torch.equal(res["ifac"][:n].cpu(), torch.from_numpy(ifac))
    f = res["fields"][:n].cpu().numpy()
    assert (f[:, 0] == 1).all() and (f[:, 8] == ctx).all() and (f[:, 36:52] == dh).all()     # ok, context, destination
    assert bool((res["status"][:n] == 0).all()) and bool((res["pt_len"][:n] == L).all())
    p, po = res["pt"].cpu().numpy(), res["pt_off"][:n].cpu().numpy()
    for i in range(n):
        assert p[po[i]:po[i] + L].tobytes() == pt[i].tobytes(), i
    # the entries past the frames carry nothing
    assert bool((res["ifac_status"][n:] == 1).all()) and bool((res["status"][n:] == 1).all())


def test_inbound_tampered_tag_fails_that_packet_alone():
    import torch
    import reticulum_amd as rt
    from reticulum_amd import pipeline
    n, L, isz = 400, 383, 16
    key, ifac_key, pt, iv, dh, ctx, ifac, t = _case(n, L, isz, 77)
    ks = rt.KeySet(key, device=0)
    framed, foff = pipeline.outbound(ks, t(pt), t(iv), t(dh), t(ctx), t(ifac), t(np.frombuffer(ifac_key, np.uint8)))
    buf = bytearray(framed[:int(foff[-1])].cpu().numpy().tobytes())
    fo = foff.cpu().numpy()
    hit = []
    for i in (3, 150, 399):
        p = int(fo[i + 1]) - 6                      # inside the last bytes of frame i: its HMAC tag
        while buf[p] in (0x7D, 0x7E) or buf[p - 1] == 0x7D or (buf[p] ^ 1) in (0x7D, 0x7E):
            p -= 1
        buf[p] ^= 1
        hit.append(i)
    res = pipeline.inbound(ks, torch.frombuffer(bytes(buf), dtype=torch.uint8).to("cuda"),
                           t(np.frombuffer(ifac_key, np.uint8)), isz, 2 * n)
    st = res["status"][:n].cpu().numpy()
    assert int(res["n_frames"]) == n
    assert sorted(np.nonzero(st)[0].tolist()) == hit and all(st[i] == 2 for i in hit)      # RT_BAD_HMAC
    assert bool((res["pt_len"][:n].cpu()[torch.from_numpy(st == 0)] == L).all())


def test_pipeline_on_a_side_stream_matches_default_stream():
    """Every stage, the torch plumbing between them included, runs on the
    stream it is given: the same batch through a side stream gives the same
    stream bytes and plaintexts as through the current stream."""
    import torch
    import reticulum_amd as rt
    from reticulum_amd import pipeline
    n, L, isz = 600, 383, 16
    key, ifac_key, pt, iv, dh, ctx, ifac, t = _case(n, L, isz, 5)
    ks = rt.KeySet(key, device=0)
    args = (t(pt), t(iv), t(dh), t(ctx), t(ifac), t(np.frombuffer(ifac_key, np.uint8)))
    framed0, foff0 = pipeline.outbound(ks, *args)
    total = int(foff0[-1])
    ref0 = pipeline.inbound(ks, framed0[:total].clone(), args[5], isz, 2 * n)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    framed1, foff1 = pipeline.outbound(ks, *args, stream=s)
    res1 = pipeline.inbound(ks, framed1[:total], args[5], isz, 2 * n, stream=s)
    s.synchronize()
    assert torch.equal(framed1[:total], framed0[:total]) and torch.equal(foff1, foff0)
    for k in ("status", "pt_len", "pt_off", "frame_pair"):
        assert torch.equal(res1[k], ref0[k]), k
    assert torch.equal(res1["ifac"][:n], ref0["ifac"][:n])      # entries past the frames are not written
    po = ref0["pt_off"][:n].cpu().numpy()
    p0, p1 = ref0["pt"].cpu().numpy(), res1["pt"].cpu().numpy()
    assert all((p0[o:o + L] == p1[o:o + L]).all() for o in po)


@pytest.mark.parametrize("n,L,isz", [(1500, 383, 16), (700, 17, 8), (257, 0, 32)])
def test_aligned_slots_change_only_offsets(n, L, isz):
    """The pipeline's own packet buffers in 128-B-aligned slots (the default,
    DESIGN.md §3) against packets packed end to end: the same HDLC stream, and
    inbound the same frames, IFACs, header fields, statuses and plaintexts;
    with slots every plaintext (and so every token's ciphertext) starts on a
    128-B line of its buffer."""
    import torch
    import reticulum_amd as rt
    from reticulum_amd import pipeline
    key, ifac_key, pt, iv, dh, ctx, ifac, t = _case(n, L, isz, 900 + n + L)
    ks = rt.KeySet(key, device=0)
    args = (t(pt), t(iv), t(dh), t(ctx), t(ifac), t(np.frombuffer(ifac_key, np.uint8)))
    fa, oa = pipeline.outbound(ks, *args, aligned=True)
    fp, op = pipeline.outbound(ks, *args, aligned=False)
    total = int(oa[-1])
    assert torch.equal(oa, op) and torch.equal(fa[:total], fp[:total])
    buf = fa[:total].clone()
    ra = pipeline.inbound(ks, buf, args[5], isz, 2 * n, aligned=True)
    rp = pipeline.inbound(ks, buf, args[5], isz, 2 * n, aligned=False)
    torch.cuda.synchronize()
    for k in ("status", "pt_len", "frame_pair", "ifac_status", "n_frames", "counts", "frame_status"):
        assert torch.equal(ra[k], rp[k]), k
    assert torch.equal(ra["frame_len"][:2 * n - 1], rp["frame_len"][:2 * n - 1])    # past the pairs: unspecified
    assert torch.equal(ra["ifac"][:n], rp["ifac"][:n]) and torch.equal(ra["fields"][:n], rp["fields"][:n])
    assert bool((ra["status"][:n] == 0).all())
    poa, pop = ra["pt_off"][:n].cpu().numpy(), rp["pt_off"][:n].cpu().numpy()
    assert ((ra["pt"].data_ptr() + poa) % 128 == 0).all()
    pa, pp = ra["pt"].cpu().numpy(), rp["pt"].cpu().numpy()
    for i in range(n):
        assert pa[poa[i]:poa[i] + L].tobytes() == pp[pop[i]:pop[i] + L].tobytes() == pt[i].tobytes(), i


def test_inbound_slots_by_default_when_padding_fits():
    """pipeline.inbound's default: slots when their padding (128 B per flag
    pair allowed) is at most the stream's size, stream offsets otherwise (a
    max_pairs sized for a stream of nothing but flags); same results both ways."""
    import torch
    import reticulum_amd as rt
    from reticulum_amd import pipeline
    n, L, isz = 1000, 383, 16
    key, ifac_key, pt, iv, dh, ctx, ifac, t = _case(n, L, isz, 4321)
    ks = rt.KeySet(key, device=0)
    ik = t(np.frombuffer(ifac_key, np.uint8))
    framed, foff = pipeline.outbound(ks, t(pt), t(iv), t(dh), t(ctx), t(ifac), ik)
    buf = framed[:int(foff[-1])].clone()
    auto = pipeline.inbound(ks, buf, ik, isz, 2 * n)
    wide = pipeline.inbound(ks, buf, ik, isz, buf.numel() // 2 + 2)
    packed = pipeline.inbound(ks, buf, ik, isz, 2 * n, aligned=False)
    torch.cuda.synchronize()
    po = auto["pt_off"][:n].cpu().numpy()
    assert ((auto["pt"].data_ptr() + po) % 128 == 0).all()                  # slots
    assert torch.equal(wide["pt_off"][:n], packed["pt_off"][:n])             # stream offsets
    assert auto["pt"].numel() > packed["pt"].numel() == wide["pt"].numel()
    for r in (auto, wide):
        assert torch.equal(r["status"][:n], packed["status"][:n]) and torch.equal(r["ifac"][:n], packed["ifac"][:n])
        p, o = r["pt"].cpu().numpy(), r["pt_off"][:n].cpu().numpy()
        assert all(p[o[i]:o[i] + L].tobytes() == pt[i].tobytes() for i in range(0, n, 7))
