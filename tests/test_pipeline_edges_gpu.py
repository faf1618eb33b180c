"""The composed inbound interface path (reticulum_amd.pipeline.inbound) on the
read loop's edge cases, checked against the oracle's composition of the
reference's steps, frame by frame:

    TCPInterface.read_loop (HDLC branch)  TCPInterface.py:387-410
    Transport.inbound, IFAC branch        Transport.py:1441-1488
    Packet.unpack                         Packet.py:242-275
    Token.decrypt                         Token.py:100-114

The stream mixes well-formed frames (made by pipeline.outbound) with junk
before the first flag, empty frames, frames too short for check_frame_len,
frames that pass it but are too short for the IFAC, frames whose IFAC flag is
cleared, frames with a corrupted IFAC, the escape sequences the two-pass
unescape treats specially (wire_vectors.json), an oversized frame and a partial
tail, so the device-side glue (frames_compact, token_spans, out_len) sees every
case the reference's loop produces.  Compared: the pairs' statuses and
lengths, the bytes the loop keeps, which frames reach Transport, the IFAC of
each, the unpack outcome and header fields, and each token's status and
plaintext.  An interface without IFAC (ifac_size 0) is covered too."""
import json
import os

import numpy as np
import pytest

from oracle import ctoken
from oracle import wire as ow

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FLAG = 0x7E


def _wire():
    with open(os.path.join(ROOT, "tests", "golden", "wire_vectors.json")) as f:
        return json.load(f)


def _edge_stream(rng, good_frames, masked_raw, good_raw, isz, hw_mtu, ifac_on):
    """good_frames: HDLC frames of valid packets; masked_raw: their IFAC-masked
    packets (to derive the flag-cleared and bad-IFAC cases; without IFAC, copies
    with the IFAC flag set); good_raw: the packets as sent."""
    wv = _wire()
    esc = next(c for c in wv["deframe"] if c["name"] == "escape edge cases")
    esc_frames = [bytes.fromhex(x) for x in esc["frames"]]
    parts = [bytes(rng.integers(0, 256, 37, dtype=np.uint8).tobytes().replace(b"\x7e", b"\x01"))]   # junk first
    k = 0
    for i, fr in enumerate(good_frames):
        parts.append(fr)
        m = i % 9
        if m == 0:
            parts.append(bytes([FLAG, FLAG]))                                 # an empty frame
        elif m == 1:
            parts.append(ow.hdlc_frame(bytes(rng.integers(0, 256, 1 + i % 19, dtype=np.uint8))))    # <= 19 B
        elif m == 2:
            short = bytes([0x80 | (i & 0x7F)]) + bytes(rng.integers(0, 256, 19 + i % (isz + 2), dtype=np.uint8))
            parts.append(ow.hdlc_frame(short))                                # passes the length check, short for IFAC
        elif m == 3:
            raw = bytearray(masked_raw[i])
            raw[0] &= 0x7F                                                    # IFAC flag cleared
            parts.append(ow.hdlc_frame(bytes(raw)))
        elif m == 4:
            raw = bytearray(masked_raw[i])
            raw[2 + (i % isz)] ^= 0x40                                        # corrupted IFAC byte
            parts.append(ow.hdlc_frame(bytes(raw)))
        elif m == 5:
            parts.append(ow.hdlc_frame(esc_frames[k % len(esc_frames)]))
            k += 1
        elif m == 6:
            parts.append(ow.hdlc_frame(bytes(rng.integers(0, 256, hw_mtu + isz + 1 + i % 7, dtype=np.uint8))))
        elif m == 7:
            raw = bytearray(masked_raw[i] if ifac_on else good_raw[i])
            raw[-1] ^= 0x01                                                   # (masked) tag byte flipped
            parts.append(ow.hdlc_frame(bytes(raw)))
    parts.append(bytes([FLAG]) + bytes(rng.integers(0, 256, 50, dtype=np.uint8).tobytes().replace(b"\x7e", b"\x02")))
    return b"".join(parts)


def _oracle_inbound(stream, key, ifac_key, isz, hw_mtu):
    frames, invalid, rest = ow.deframe(stream, hw_mtu, isz)
    out = []
    for fr in frames:
        rec = {"frame": fr}
        if isz:
            r = ow.ifac_unmask(fr, isz, ifac_key)
        else:
            r = None if (len(fr) <= 2 or fr[0] & 0x80) else (b"", fr)
        rec["ifac_ok"] = r is not None
        if r is not None:
            rec["ifac"], new_raw = r
            f = ow.unpack(new_raw)
            rec["unpack"] = f
            if f is not None:
                rec["token"] = ctoken.decrypt(key, f["data"])
        out.append(rec)
    return out, invalid, rest


def _check(res, stream, key, ifac_key, isz, hw_mtu):
    import torch
    torch.cuda.synchronize()
    recs, invalid, rest = _oracle_inbound(stream, key, ifac_key, isz, hw_mtu)
    pairs, consumed = (int(x) for x in res["counts"].cpu())
    assert stream[consumed:] == rest
    st = res["frame_status"][:pairs].cpu().numpy()
    assert int(res["n_frames"]) == len(recs) == int((st == 0).sum())
    fp = res["frame_pair"][:len(recs)].cpu().numpy()
    assert (st[fp] == 0).all() and (np.diff(fp) > 0).all()
    ist = res["ifac_status"].cpu().numpy()
    fields = res["fields"].cpu().numpy()
    tst = res["status"].cpu().numpy()
    pl, po = res["pt_len"].cpu().numpy(), res["pt_off"].cpu().numpy()
    pt = res["pt"].cpu().numpy()
    ifac = res["ifac"].cpu().numpy()
    seen = {"ifac_drop": 0, "unpack_fail": 0, "tok_fail": 0, "ok": 0}
    for i, r in enumerate(recs):
        assert (ist[i] == 0) == r["ifac_ok"], i
        if not r["ifac_ok"]:
            seen["ifac_drop"] += 1
            assert fields[i, 0] == 0 and tst[i] == 1, i      # nothing reaches unpack: TOO_SHORT span
            continue
        assert ifac[i].tobytes() == r["ifac"], i
        f = r["unpack"]
        assert bool(fields[i, 0]) == (f is not None), i
        if f is None:
            seen["unpack_fail"] += 1
            assert tst[i] == 1, i
            continue
        assert fields[i, 1] == f["flags"] and fields[i, 2] == f["hops"] and fields[i, 8] == f["context"], i
        assert fields[i, 36:52].tobytes() == f["destination_hash"], i
        assert fields[i, 52:84].tobytes() == f["packet_hash"], i
        s, p = r["token"]
        assert tst[i] == s, (i, tst[i], s)
        if s == 0:
            seen["ok"] += 1
            assert pt[po[i]:po[i] + pl[i]].tobytes() == p, i
        else:
            seen["tok_fail"] += 1
    # past the frames: nothing
    assert (ist[len(recs):] == 1).all() and (tst[len(recs):] == 1).all()
    return seen, invalid


@pytest.mark.parametrize("aligned", [False, True])
@pytest.mark.parametrize("isz", [32, 16, 0])
def test_inbound_edge_cases_match_the_oracle_composition(isz, aligned):
    import torch
    import reticulum_amd as rt
    from reticulum_amd import pipeline
    rng = np.random.Generator(np.random.PCG64(900 + isz))
    n, L, hw_mtu = 180, 383, 1000
    key = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
    ifac_key = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
    pt = rng.integers(0, 256, (n, L), dtype=np.uint8)
    iv = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    dh = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    ctx = rng.integers(0, 256, n, dtype=np.uint8)
    ifac = rng.integers(0, 256, (n, isz), dtype=np.uint8)
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)     # noqa: E731
    ks = rt.KeySet(key, device=0)
    ik = t(np.frombuffer(ifac_key, np.uint8))
    framed, foff = pipeline.outbound(ks, t(pt), t(iv), t(dh), t(ctx), t(ifac) if isz else None, ik)
    fo = foff.cpu().numpy()
    fb = framed[:int(fo[-1])].cpu().numpy().tobytes()
    good = [fb[fo[i]:fo[i + 1]] for i in range(n)]
    masked, sent = [], []
    for i in range(n):
        raw = ow.pack_header(0, 0, dh[i].tobytes(), int(ctx[i])) + ctoken.encrypt(key, iv[i].tobytes(), pt[i].tobytes())
        m = ow.ifac_mask(raw, ifac[i].tobytes(), ifac_key) if isz else raw
        assert ow.hdlc_frame(m) == good[i]
        sent.append(m)
        masked.append(m if isz else bytes([raw[0] | 0x80]) + raw[1:])     # no IFAC: flagged copies must be dropped
    stream = _edge_stream(rng, good, masked, sent, max(isz, 1), hw_mtu, isz > 0)
    buf = torch.frombuffer(bytearray(stream), dtype=torch.uint8).to(dev)
    res = pipeline.inbound(ks, buf, ik, isz, len(stream) // 2 + 2, hw_mtu=hw_mtu, aligned=aligned)
    seen, invalid = _check(res, stream, key, ifac_key, isz, hw_mtu)
    # every case was exercised
    assert invalid and seen["ifac_drop"] and seen["ok"] >= n and seen["tok_fail"], seen
    pairs = int(res["counts"][0])
    st = res["frame_status"][:pairs].cpu().numpy()
    ln = res["frame_len"][:pairs].cpu().numpy()
    assert (st == 2).any()                                      # empty frames skipped
    assert sorted(ln[st == 1].tolist()) == sorted(invalid)


@pytest.mark.parametrize("aligned", [False, True])
def test_inbound_reads_split_across_calls_keep_the_loops_buffer(aligned):
    """Two reads: the bytes the first leaves (counts[1] onwards, a partial
    frame) are carried into the second, as the read loop keeps them in its
    buffer; the frames of both reads together are the oracle's."""
    import torch
    import reticulum_amd as rt
    from reticulum_amd import pipeline
    rng = np.random.Generator(np.random.PCG64(31))
    n, L, isz = 64, 100, 16
    key = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
    ifac_key = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)     # noqa: E731
    pt = rng.integers(0, 256, (n, L), dtype=np.uint8)
    args = [t(pt)] + [t(rng.integers(0, 256, s, dtype=np.uint8)) for s in ((n, 16), (n, 16), (n,), (n, isz))]
    ks = rt.KeySet(key, device=0)
    ik = t(np.frombuffer(ifac_key, np.uint8))
    framed, foff = pipeline.outbound(ks, *args, ik)
    stream = framed[:int(foff[-1])].cpu().numpy().tobytes()
    cut = int(foff[n // 2]) + 37                     # inside frame n/2
    got = []
    carry = b""
    for chunk in (stream[:cut], stream[cut:]):
        data = carry + chunk
        res = pipeline.inbound(ks, torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev), ik, isz,
                               len(data) // 2 + 2, aligned=aligned)
        torch.cuda.synchronize()
        nf = int(res["n_frames"])
        po, pl = res["pt_off"][:nf].cpu().numpy(), res["pt_len"][:nf].cpu().numpy()
        p = res["pt"].cpu().numpy()
        assert bool((res["status"][:nf] == 0).all())
        got += [p[o:o + k].tobytes() for o, k in zip(po, pl)]
        carry = data[int(res["counts"][1]):]
    assert got == [pt[i].tobytes() for i in range(n)]


@pytest.mark.parametrize("aligned", [False, True])
@pytest.mark.parametrize("isz", [0, 16])
def test_inbound_empty_read(isz, aligned):
    """A zero-byte read (the read loop's empty recv) through the whole inbound
    path: no frames, nothing consumed, every entry empty (the
    no-IFAC branch gathered each entry's flag byte from an empty buffer)."""
    import torch
    import reticulum_amd as rt
    from reticulum_amd import pipeline
    dev = torch.device("cuda", 0)
    ks = rt.KeySet(bytes(range(64)), device=0)
    ik = torch.arange(64, dtype=torch.uint8, device=dev)
    res = pipeline.inbound(ks, torch.empty(0, dtype=torch.uint8, device=dev), ik, isz, 4, aligned=aligned)
    torch.cuda.synchronize()
    assert int(res["n_frames"]) == 0
    assert res["counts"].cpu().tolist() == [0, 0]
    assert (res["ifac_status"].cpu() == 1).all()
    assert (res["status"].cpu() == 1).all()
    assert (res["pt_len"].cpu() == 0).all()


@pytest.mark.parametrize("phase", [0, 35, 127])
def test_deframe_slots_match_stream_offsets(phase):
    """rt_hdlc_deframe_slots against rt_hdlc_deframe on the edge-case stream
    (junk, empty and oversized frames, escapes): the same pairs, lengths,
    statuses, consumed bytes and frame bytes; each frame's byte `phase` on a
    128-B line; frames disjoint inside the documented capacity."""
    import torch
    from reticulum_amd import device
    rng = np.random.Generator(np.random.PCG64(77 + phase))
    ow_frames = [ow.hdlc_frame(rng.integers(0, 256, int(rng.integers(1, 700)), dtype=np.uint8).tobytes())
                 for _ in range(300)]
    parts = []
    for f in ow_frames:
        r = rng.random()
        parts.append(f if r > 0.1 else (b"\x7e\x7e" + f if r > 0.05 else f[:-1]))
    stream = bytes(rng.integers(0, 256, 50, dtype=np.uint8)) + b"".join(parts) + b"\x7d\x5e\x7e\x7d"
    dev = torch.device("cuda", 0)
    buf = torch.frombuffer(bytearray(stream), dtype=torch.uint8).to(dev)
    mp = len(stream) // 2 + 2
    res = []
    for ph in (None, phase):
        out = torch.zeros(device.deframe_slots_bytes(buf.numel(), mp) if ph is not None else buf.numel(),
                          dtype=torch.uint8, device=dev)
        fo = torch.empty(mp, dtype=torch.int64, device=dev)
        fl = torch.empty(mp, dtype=torch.int32, device=dev)
        st = torch.full((mp,), -1, dtype=torch.int32, device=dev)
        ct = torch.empty(2, dtype=torch.int64, device=dev)
        device.hdlc_deframe(buf, out, fo, fl, st, ct, hw_mtu=500, ifac_size=0, line_phase=ph)
        torch.cuda.synchronize()
        res.append((out, fo.cpu().numpy(), fl.cpu().numpy(), st.cpu().numpy(), ct.cpu().tolist()))
    (o0, f0, l0, s0, c0), (o1, f1, l1, s1, c1) = res
    pairs = c0[0]
    assert c0 == c1 and pairs > 300
    assert (l0[:pairs] == l1[:pairs]).all() and (s0[:pairs] == s1[:pairs]).all()
    b0, b1 = o0.cpu().numpy(), o1.cpu().numpy()
    ends = []
    for k in range(pairs):
        assert b0[f0[k]:f0[k] + l0[k]].tobytes() == b1[f1[k]:f1[k] + l1[k]].tobytes(), k
        assert (o1.data_ptr() + int(f1[k]) + phase) % 128 == 0, k
        ends.append((int(f1[k]), int(f1[k]) + int(l1[k])))
    assert all(a[1] <= b[0] for a, b in zip(ends, ends[1:])) and ends[-1][1] <= o1.numel()
