"""Wire-side neighbours: HDLC framing / deframing
(TCPInterface.py:44-53, 323, 387-410), IFAC mask / unmask (Transport.py:
1069-1101, 1441-1475), Packet unpack / hash / header pack (Packet.py:
167-268, 342-353).

CPU: the oracle (oracle/wire.py) against fixtures produced by the
reference's own code (tests/golden/gen_wire.py: HDLC.escape, the real
TCPClientInterface.read_loop over a fake socket, Transport.transmit /
inbound with a real Ed25519 identity, Packet.unpack / pack).
GPU (-m gpu): the wire kernels through the C-ABI, bit-exact against the same
fixtures and against the oracle on random batches.
"""
import importlib.util
import json
import os

import numpy as np
import pytest

from oracle import wire as ow
from tests_helpers import b

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def wv():
    with open(os.path.join(HERE, "golden", "wire_vectors.json")) as f:
        return json.load(f)


def _oversized_body():
    spec = importlib.util.spec_from_file_location("gen_wire", os.path.join(HERE, "golden", "gen_wire.py"))
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    return g.oversized_body()


def _stream(r):
    return b(r["stream"]) if r["stream"] is not None else b"\x7e" + _oversized_body() + b(r["stream_tail"])


def _h(x):
    return None if x is None else b(x)


# ------------------------------------------------------------------ oracle --

def test_oracle_escape(wv):
    for e in wv["escape"]:
        assert ow.hdlc_escape(b(e["data"])).hex() == e["escaped"]


def test_oracle_deframe_matches_reference_read_loop(wv):
    for r in wv["deframe"]:
        frames, invalid, _ = ow.deframe(_stream(r), r["hw_mtu"], r["ifac_size"])
        assert [f.hex() for f in frames] == r["frames"], r["name"]
        assert invalid == r["invalid"], r["name"]
    c = wv["deframe_chunked"]
    buf, got = b"", []
    for ch in c["chunks"]:
        fr, _, buf = ow.deframe(buf + b(ch))
        got += fr
    assert [f.hex() for f in got] == c["frames"]


def test_oracle_lone_flag_across_reads(wv):
    """Junk then a lone flag: the read loop keeps the whole buffer, or drops
    all of it past 2*HW_MTU (fixtures from the reference's read loop)."""
    for r in wv["deframe_lone_flag"]:
        buf, got = b"", []
        for ch in r["chunks"]:
            fr, _, buf = ow.deframe(buf + b(ch), r["hw_mtu"])
            got += fr
        assert [f.hex() for f in got] == r["frames"], r["name"]


def test_oracle_ifac(wv):
    for r in wv["ifac"]:
        m = ow.ifac_mask(b(r["raw"]), b(r["ifac"]), b(r["ifac_key"]))
        assert m.hex() == r["masked"]
        ifac, new_raw = ow.ifac_unmask(m, r["ifac_size"], b(r["ifac_key"]))
        assert ifac.hex() == r["ifac"] and new_raw.hex() == r["inbound_reassembled"] == r["raw"]


def test_oracle_unpack_and_pack(wv):
    for r in wv["unpack"]:
        u = ow.unpack(b(r["raw"]))
        assert (u is not None) == r["ok"], r["raw"][:8]
        if u:
            for k in ("header_type", "context_flag", "transport_type", "destination_type", "packet_type", "hops",
                      "flags", "context"):
                assert u[k] == r[k], k
            assert u["data"].hex() == r["data"] and u["packet_hash"].hex() == r["packet_hash"]
            assert u["destination_hash"].hex() == r["destination_hash"]
            assert (None if u["transport_id"] is None else u["transport_id"].hex()) == r["transport_id"]
    for r in wv["pack"]:
        h = ow.pack_header(r["flags"], r["hops"], b(r["destination_hash"]), r["context"], _h(r["transport_id"]))
        assert (h + b(r["data"])).hex() == r["raw"]
        assert ow.unpack(b(r["raw"]))["packet_hash"].hex() == r["packet_hash"]


# --------------------------------------------------------------------- GPU --

@pytest.mark.gpu
def test_gpu_escape_and_frame(wv):
    from reticulum_amd import wire
    for e in wv["escape"]:
        assert wire.HDLC.escape(b(e["data"])).hex() == e["escaped"]
    rng = np.random.Generator(np.random.PCG64(323))
    pk = []
    for n in rng.integers(0, 700, 2000):
        a = rng.integers(0, 256, int(n), dtype=np.uint8)
        a[rng.random(int(n)) < 0.1] = 0x7E
        a[rng.random(int(n)) < 0.1] = 0x7D
        pk.append(a.tobytes())
    stream, off = wire.hdlc_frame_batch(pk)
    assert stream == b"".join(ow.hdlc_frame(p) for p in pk)
    assert all(stream[int(off[i]):int(off[i + 1])] == ow.hdlc_frame(p) for i, p in enumerate(pk[:50]))


@pytest.mark.gpu
def test_gpu_deframe_matches_reference_read_loop(wv):
    from reticulum_amd import wire
    for r in wv["deframe"]:
        frames, invalid, consumed = wire.deframe(_stream(r), r["hw_mtu"], r["ifac_size"] or 0)
        assert [f.hex() for f in frames] == r["frames"], r["name"]
        assert invalid == r["invalid"], r["name"]
        _, _, rest = ow.deframe(_stream(r), r["hw_mtu"], r["ifac_size"])
        assert _stream(r)[consumed:] == rest, r["name"]
    c = wv["deframe_chunked"]
    d = wire.Deframer()
    got = []
    for ch in c["chunks"]:
        got += d.feed(b(ch))
    assert [f.hex() for f in got] == c["frames"]


@pytest.mark.gpu
def test_gpu_lone_flag_across_reads(wv):
    from reticulum_amd import wire
    for r in wv["deframe_lone_flag"]:
        d = wire.Deframer(hw_mtu=r["hw_mtu"])
        got = []
        for ch in r["chunks"]:
            got += d.feed(b(ch))
        assert [f.hex() for f in got] == r["frames"], r["name"]


@pytest.mark.gpu
def test_gpu_frame_deframe_roundtrip_large():
    """Size-independent property: 20 000 framed packets deframe to themselves."""
    from reticulum_amd import wire
    rng = np.random.Generator(np.random.PCG64(410))
    pk = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in rng.integers(20, 520, 20000)]
    stream, _ = wire.hdlc_frame_batch(pk)
    frames, invalid, consumed = wire.deframe(stream)
    assert frames == pk and invalid == [] and consumed == len(stream) - 1


@pytest.mark.gpu
def test_gpu_ifac(wv):
    from reticulum_amd import wire
    for size in (8, 16):
        rs = [r for r in wv["ifac"] if r["ifac_size"] == size]
        key = b(rs[0]["ifac_key"])
        masked = wire.ifac_mask_batch([b(r["raw"]) for r in rs], [b(r["ifac"]) for r in rs], key)
        assert [m.hex() for m in masked] == [r["masked"] for r in rs]
        un = wire.ifac_unmask_batch(masked, size, key)
        assert [(i.hex(), p.hex()) for i, p in un] == [(r["ifac"], r["inbound_reassembled"]) for r in rs]
    # random batch vs the oracle, with packets the reference drops before signing
    rng = np.random.Generator(np.random.PCG64(1101))
    key = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
    raws = [rng.integers(0, 128, 2, dtype=np.uint8).tobytes() + rng.integers(0, 256, int(n), dtype=np.uint8).tobytes()
            for n in rng.integers(0, 600, 500)]
    ifacs = [rng.integers(0, 256, 16, dtype=np.uint8).tobytes() for _ in raws]
    masked = wire.ifac_mask_batch(raws, ifacs, key)
    assert masked == [ow.ifac_mask(r, f, key) for r, f in zip(raws, ifacs)]
    probes = masked + [bytes([0x05]) + m[1:] for m in masked[:20]] + [m[:18] for m in masked[:20]] + [b"\x80\x01"]
    got = wire.ifac_unmask_batch(probes, 16, key)
    assert got == [ow.ifac_unmask(p, 16, key) for p in probes]


@pytest.mark.gpu
def test_gpu_unpack_and_pack(wv):
    from reticulum_amd import wire
    raws = [b(r["raw"]) for r in wv["unpack"]]
    got = wire.unpack_batch(raws)
    for r, g in zip(wv["unpack"], got):
        assert (g is not None) == r["ok"], r["raw"][:8]
        if g:
            assert g["packet_hash"].hex() == r["packet_hash"] and g["data"].hex() == r["data"]
            assert g["destination_hash"].hex() == r["destination_hash"] and g["context"] == r["context"]
            assert (None if g["transport_id"] is None else g["transport_id"].hex()) == r["transport_id"]
            for k in ("header_type", "context_flag", "transport_type", "destination_type", "packet_type", "hops"):
                assert g[k] == r[k], k
    for ht in (0, 1):
        rs = [r for r in wv["pack"] if (r["transport_id"] is not None) == bool(ht)]
        hdrs = wire.pack_headers_batch([r["flags"] for r in rs], [r["hops"] for r in rs],
                                       [b(r["destination_hash"]) for r in rs], [r["context"] for r in rs],
                                       [b(r["transport_id"]) for r in rs] if ht else None)
        assert [(h + b(r["data"])).hex() for h, r in zip(hdrs, rs)] == [r["raw"] for r in rs]
    rng = np.random.Generator(np.random.PCG64(268))
    raws = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in rng.integers(0, 520, 3000)]
    got = wire.unpack_batch(raws)
    for raw, g in zip(raws, got):
        o = ow.unpack(raw)
        assert (g is None) == (o is None)
        if g:
            assert g == {k: o[k] for k in g}


@pytest.mark.gpu
def test_gpu_device_forms_match_host_forms():
    """reticulum_amd.device's tensor entry points give what the host
    conveniences (and so the oracle) give, on one random batch."""
    import torch
    from reticulum_amd import device, wire
    rng = np.random.Generator(np.random.PCG64(228))
    pk = [rng.integers(0, 128, 2, dtype=np.uint8).tobytes() + rng.integers(0, 256, int(n), dtype=np.uint8).tobytes()
          for n in rng.integers(30, 600, 700)]
    lens = np.array([len(p) for p in pk], np.int32)
    off = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.int64)
    dev = torch.device("cuda", 0)
    flat = torch.from_numpy(np.frombuffer(b"".join(pk), np.uint8).copy()).to(dev)
    t_off, t_len = torch.from_numpy(off).to(dev), torch.from_numpy(lens).to(dev)
    n = len(pk)
    # framing, then deframing the stream
    framed = torch.empty(int(2 * lens.sum() + 2 * n), dtype=torch.uint8, device=dev)
    foff = torch.empty(n + 1, dtype=torch.int64, device=dev)
    device.hdlc_frame(flat, t_off, t_len, framed, foff)
    total = int(foff[-1])
    host_stream, _ = wire.hdlc_frame_batch(pk)
    assert framed[:total].cpu().numpy().tobytes() == host_stream
    buf = framed[:total].clone()
    pairs = 2 * n
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    d_off = torch.empty(pairs, dtype=torch.int64, device=dev)
    d_len = torch.empty(pairs, dtype=torch.int32, device=dev)
    d_st = torch.empty(pairs, dtype=torch.int32, device=dev)
    cnt = torch.empty(2, dtype=torch.int64, device=dev)
    device.hdlc_deframe(buf, out, d_off, d_len, d_st, cnt)
    o, dl, ds = out.cpu().numpy().tobytes(), d_len.cpu().numpy(), d_st.cpu().numpy()
    do = d_off.cpu().numpy()
    k = int(cnt[0])
    frames = [o[int(do[i]):int(do[i]) + int(dl[i])] for i in range(k) if ds[i] == wire.FRAME_OK]
    assert frames == [p for p in pk if len(p) > 19] and int(cnt[1]) == total - 1
    # IFAC mask / unmask
    key_h = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
    ifacs = rng.integers(0, 256, (n, 8), dtype=np.uint8)
    key = torch.from_numpy(np.frombuffer(key_h, np.uint8).copy()).to(dev)
    ti = torch.from_numpy(ifacs).to(dev)
    m_len = lens + 8
    m_off = np.concatenate([[0], np.cumsum(m_len[:-1])]).astype(np.int64)
    masked = torch.empty(int(m_len.sum()), dtype=torch.uint8, device=dev)
    tm_off, tm_len = torch.from_numpy(m_off).to(dev), torch.from_numpy(m_len).to(dev)
    device.ifac_mask(flat, t_off, t_len, ti, key, masked, tm_off)
    mh = masked.cpu().numpy().tobytes()
    got = [mh[int(a):int(a) + int(b)] for a, b in zip(m_off, m_len)]
    assert got == wire.ifac_mask_batch(pk, [r.tobytes() for r in ifacs], key_h)
    un = torch.empty_like(masked)
    i_out = torch.empty((n, 8), dtype=torch.uint8, device=dev)
    ust = torch.empty(n, dtype=torch.int32, device=dev)
    device.ifac_unmask(masked, tm_off, tm_len, key, i_out, un, tm_off, ust)
    uh = un.cpu().numpy().tobytes()
    assert (ust.cpu().numpy() == 0).all() and torch.equal(i_out, ti)
    assert [uh[int(a):int(a) + int(b)] for a, b in zip(m_off, lens)] == [bytes([p[0] & 0x7F]) + p[1:] for p in pk]
    # out_len: the unmasked length where the IFAC checks pass, 0 where the
    # packet is dropped (here: every third one cut to 2 + ifac_size bytes)
    short = tm_len.clone()
    short[::3] = 10
    o_len = torch.full((n,), 7, dtype=torch.int32, device=dev)
    device.ifac_unmask(masked, tm_off, short, key, i_out, un, tm_off, ust, out_len=o_len)
    drop = np.arange(n) % 3 == 0
    assert np.array_equal(ust.cpu().numpy(), drop.astype(np.int32))
    assert np.array_equal(o_len.cpu().numpy(), np.where(drop, 0, lens).astype(np.int32))
    # unpack
    fields = torch.empty((n, 96), dtype=torch.uint8, device=dev)
    device.packet_unpack(flat, t_off, t_len, fields)
    f = fields.cpu().numpy().view(wire.FIELDS_DTYPE).reshape(-1)
    ref = wire.unpack_batch(pk)
    for i in range(n):
        assert bool(f[i]["ok"]) == (ref[i] is not None)
        if ref[i]:
            assert bytes(f[i]["packet_hash"]) == ref[i]["packet_hash"]


@pytest.mark.gpu
@pytest.mark.parametrize("density", [0.0, 0.02, 0.3, 0.9])
def test_gpu_deframe_escape_dense_writes_only_frames(density):
    """Framing's and unescape's row-wide 16-B stores (a lane stores its own
    bytes and then its neighbour's first ones, which the neighbour stores
    too): the framed stream equals the oracle's, and frames of
    0-700 B whose bytes are 7E/7D with the given probability (lanes with many
    escapes keep as few as 8 of their 16 bytes) come back exact, and no byte of
    the output buffer outside the frames' own output is written."""
    import torch
    from reticulum_amd import device, wire
    rng = np.random.Generator(np.random.PCG64(int(density * 1000) + 7))
    pk = []
    for n in rng.integers(0, 700, 3000):
        a = rng.integers(0, 256, int(n), dtype=np.uint8)
        hit = rng.random(int(n)) < density
        a[hit] = rng.choice(np.array([0x7E, 0x7D], np.uint8), int(hit.sum()))
        pk.append(a.tobytes())
    stream, _ = wire.hdlc_frame_batch(pk)
    # the framing side of the same row-wide stores: the stream is the reference's escape of every packet
    assert stream == b"".join(ow.hdlc_frame(p) for p in pk)
    dev = torch.device("cuda", 0)
    buf = torch.from_numpy(np.frombuffer(stream, np.uint8).copy()).to(dev)
    total = len(stream)
    pairs = 2 * len(pk)
    out = torch.full((total,), 0xA5, dtype=torch.uint8, device=dev)
    d_off = torch.empty(pairs, dtype=torch.int64, device=dev)
    d_len = torch.empty(pairs, dtype=torch.int32, device=dev)
    d_st = torch.empty(pairs, dtype=torch.int32, device=dev)
    cnt = torch.empty(2, dtype=torch.int64, device=dev)
    device.hdlc_deframe(buf, out, d_off, d_len, d_st, cnt)
    o = out.cpu().numpy()
    k = int(cnt[0])
    do, dl, ds = d_off.cpu().numpy()[:k], d_len.cpu().numpy()[:k], d_st.cpu().numpy()[:k]
    frames = [o[int(do[i]):int(do[i]) + int(dl[i])].tobytes() for i in range(k) if ds[i] == wire.FRAME_OK]
    assert frames == [p for p in pk if len(p) > 19]
    written = np.zeros(total, bool)
    for i in range(k):
        written[int(do[i]):int(do[i]) + int(dl[i])] = True
    assert (o[~written] == 0xA5).all()
