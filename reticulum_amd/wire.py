"""Wire-side neighbours of the token path on the GPU.

* ``HDLC.escape`` / ``hdlc_frame_batch``   TCPInterface.py:44-53, :323
* ``Deframer``                              the HDLC read loop, TCPInterface.py:387-410, :336-339
* ``ifac_mask_batch`` / ``ifac_unmask_batch``  Transport.py:1069-1101 / :1441-1475
  (the Ed25519 signature that yields the IFAC stays with the caller)
* ``unpack_batch``                          Packet.unpack + get_hash, Packet.py:236-268, 342-353
* ``pack_headers_batch``                    Packet.pack's header, Packet.py:167-228

Host-buffer conveniences over librnstok's device kernels (wire_kernels.hip);
``reticulum_amd.device`` has the device-resident forms (hdlc_frame, hdlc_deframe,
ifac_mask, ifac_unmask, packet_unpack, pack_headers).  No CPU fallback.
"""
import ctypes

import numpy as np

from . import _native

FLAG, ESC, ESC_MASK = 0x7E, 0x7D, 0x20
HW_MTU = 262144                      # TCPInterface.HW_MTU
FRAME_OK, FRAME_BAD_LEN, FRAME_EMPTY = 0, 1, 2


class PacketFields(ctypes.Structure):
    """rt_packet_fields (include/rnstok.h)."""
    _fields_ = [("ok", ctypes.c_uint8), ("flags", ctypes.c_uint8), ("hops", ctypes.c_uint8),
                ("header_type", ctypes.c_uint8), ("context_flag", ctypes.c_uint8),
                ("transport_type", ctypes.c_uint8), ("destination_type", ctypes.c_uint8),
                ("packet_type", ctypes.c_uint8), ("context", ctypes.c_uint8), ("reserved", ctypes.c_uint8 * 3),
                ("data_offset", ctypes.c_uint32), ("data_len", ctypes.c_uint32),
                ("transport_id", ctypes.c_uint8 * 16), ("destination_hash", ctypes.c_uint8 * 16),
                ("packet_hash", ctypes.c_uint8 * 32), ("reserved2", ctypes.c_uint8 * 12)]


FIELDS_DTYPE = np.dtype([("ok", "u1"), ("flags", "u1"), ("hops", "u1"), ("header_type", "u1"),
                         ("context_flag", "u1"), ("transport_type", "u1"), ("destination_type", "u1"),
                         ("packet_type", "u1"), ("context", "u1"), ("reserved", "u1", 3), ("data_offset", "<u4"),
                         ("data_len", "<u4"), ("transport_id", "u1", 16), ("destination_hash", "u1", 16),
                         ("packet_hash", "u1", 32), ("reserved2", "u1", 12)])
assert FIELDS_DTYPE.itemsize == ctypes.sizeof(PacketFields) == 96


class _Dev:
    """Device scratch for the host conveniences: upload numpy arrays, run,
    download, free (through the library's own allocation helpers)."""

    def __init__(self, device=None):
        self.lib = _native.load()
        self.ctx = _native.context(device)
        self.bufs = []
        self.keep = []          # host arrays an enqueued copy may still read

    def alloc(self, nbytes):
        p = self.lib.rt_device_alloc(self.ctx, max(int(nbytes), 1))
        if not p:
            raise _native.NativeError(_native.RT_E_NOMEM, _native.last_error())
        self.bufs.append(p)
        return p

    def up(self, arr):
        if arr is None:
            return None
        arr = np.ascontiguousarray(arr)
        p = self.alloc(arr.nbytes)
        if arr.nbytes:
            _native.check(self.lib.rt_memcpy_h2d(self.ctx, p, arr.ctypes.data_as(ctypes.c_void_p), arr.nbytes, None))
            self.keep.append(arr)
        return p

    def down(self, p, arr):
        """Copy device bytes into arr and wait for them: the copy is an async
        copy on the null stream, which HIP does not promise to complete
        before returning for pageable memory."""
        if arr.nbytes:
            _native.check(self.lib.rt_memcpy_d2h(self.ctx, arr.ctypes.data_as(ctypes.c_void_p), p, arr.nbytes, None))
            self.sync()
        return arr

    def sync(self):
        _native.check(self.lib.rt_stream_sync(self.ctx, None))

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.sync()
        self.keep = []
        for p in self.bufs:
            self.lib.rt_device_free(self.ctx, p)
        self.bufs = []


def _pack(items):
    items = [bytes(x) for x in items]
    lens = np.array([len(x) for x in items], np.uint32)
    off = np.zeros(len(items), np.uint64)
    if len(items) > 1:
        off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    buf = np.frombuffer(b"".join(items), np.uint8) if items and lens.sum() else np.zeros(1, np.uint8)
    return buf, off, lens


def _check_bytes(x, what):
    if not isinstance(x, (bytes, bytearray, memoryview)):
        raise TypeError(f"{what} must be bytes")


# ------------------------------------------------------------------- HDLC --

def hdlc_frame_batch(packets, device=None):
    """Frames for many packets in one stream: returns (stream bytes, frame
    offsets (n+1,)), frame i = stream[off[i]:off[i+1]] = 7E || escape || 7E
    (process_outgoing, TCPInterface.py:323)."""
    for p in packets:
        _check_bytes(p, "packet")
    n = len(packets)
    if n == 0:
        return b"", np.zeros(1, np.uint64)
    buf, off, lens = _pack(packets)
    cap = int(2 * lens.astype(np.uint64).sum() + 2 * n)
    with _Dev(device) as d:
        lib = d.lib
        p_buf, p_off, p_len = d.up(buf), d.up(off), d.up(lens)
        p_out = d.alloc(cap)
        p_foff = d.alloc(8 * (n + 1))
        ws = d.alloc(lib.rt_hdlc_frame_workspace_bytes(n))
        _native.check(lib.rt_hdlc_frame(d.ctx, p_buf, p_off, p_len, n, p_out, p_foff, ws, None))
        foff = d.down(p_foff, np.zeros(n + 1, np.uint64))
        out = d.down(p_out, np.zeros(int(foff[-1]), np.uint8))
    return out.tobytes(), foff


class HDLC:
    """RNS.Interfaces.TCPInterface.HDLC with the escape on the GPU."""
    FLAG = FLAG
    ESC = ESC
    ESC_MASK = ESC_MASK

    @staticmethod
    def escape(data, device=None):
        _check_bytes(data, "data")
        if not data:
            return b""
        stream, _ = hdlc_frame_batch([bytes(data)], device)
        return stream[1:-1]


class Deframer:
    """The HDLC read loop of TCPClientInterface (TCPInterface.py:387-410) over
    a byte stream: ``feed(data)`` returns the frames the loop hands to
    process_incoming for that read; frames dropped by check_frame_len are
    appended to ``invalid`` (their lengths).  The unconsumed tail is kept, as
    the loop keeps frame_buffer."""

    def __init__(self, hw_mtu=HW_MTU, ifac_size=None, device=None):
        self.hw_mtu, self.ifac_size, self.device = hw_mtu, ifac_size or 0, device
        self.buffer = b""
        self.invalid = []

    def feed(self, data):
        _check_bytes(data, "data")
        self.buffer += bytes(data)
        frames, invalid, consumed = deframe(self.buffer, self.hw_mtu, self.ifac_size, self.device)
        self.invalid += invalid
        self.buffer = self.buffer[consumed:]
        return frames


def deframe(buf, hw_mtu=HW_MTU, ifac_size=0, device=None):
    """One pass of the read loop over ``buf``: (frames, invalid_lengths,
    bytes_consumed)."""
    n = len(buf)
    if n == 0:
        return [], [], 0
    max_pairs = buf.count(bytes([FLAG]))
    arr = np.frombuffer(bytes(buf), np.uint8)
    with _Dev(device) as d:
        lib = d.lib
        p_buf = d.up(arr)
        p_out = d.alloc(n)
        p_off = d.alloc(8 * max(max_pairs, 1))
        p_len = d.alloc(4 * max(max_pairs, 1))
        p_st = d.alloc(4 * max(max_pairs, 1))
        p_cnt = d.alloc(16)
        ws = d.alloc(lib.rt_hdlc_deframe_workspace_bytes(n))
        _native.check(lib.rt_hdlc_deframe(d.ctx, p_buf, n, hw_mtu, ifac_size or 0, p_out, p_off, p_len, p_st, p_cnt,
                                          max_pairs, ws, None))
        counts = d.down(p_cnt, np.zeros(2, np.uint64))
        k = int(counts[0])
        off = d.down(p_off, np.zeros(max(max_pairs, 1), np.uint64))[:k]
        ln = d.down(p_len, np.zeros(max(max_pairs, 1), np.uint32))[:k]
        st = d.down(p_st, np.zeros(max(max_pairs, 1), np.int32))[:k]
        out = d.down(p_out, np.zeros(n, np.uint8)).tobytes()
    frames = [out[int(o):int(o) + int(l)] for o, l, s in zip(off, ln, st) if s == FRAME_OK]
    invalid = [int(l) for l, s in zip(ln, st) if s == FRAME_BAD_LEN]
    return frames, invalid, int(counts[1])


# ------------------------------------------------------------------- IFAC --

def ifac_mask_batch(raws, ifacs, ifac_key, device=None):
    """Transport.transmit's IFAC step for many packets: raws[i] with its
    access code ifacs[i] (sign(raw)[-ifac_size:], from the caller) -> the
    masked packet handed to process_outgoing."""
    n = len(raws)
    if n == 0:
        return []
    size = len(ifacs[0])
    if any(len(f) != size for f in ifacs) or len(ifacs) != n:
        raise ValueError("one IFAC of equal size per packet")
    if any(len(r) < 2 for r in raws):
        raise ValueError("packets need the 2 header bytes")
    buf, off, lens = _pack(raws)
    out_len = lens.astype(np.uint64) + size
    out_off = np.zeros(n, np.uint64)
    out_off[1:] = np.cumsum(out_len[:-1])
    key = np.frombuffer(bytes(ifac_key), np.uint8)
    with _Dev(device) as d:
        p_out = d.alloc(int(out_len.sum()))
        _native.check(d.lib.rt_ifac_mask(d.ctx, d.up(buf), d.up(off), d.up(lens),
                                         d.up(np.frombuffer(b"".join(bytes(f) for f in ifacs), np.uint8)), size,
                                         d.up(key), len(key), p_out, d.up(out_off), n, None))
        out = d.down(p_out, np.zeros(int(out_len.sum()), np.uint8)).tobytes()
    return [out[int(o):int(o) + int(l)] for o, l in zip(out_off, out_len)]


def ifac_unmask_batch(raws, ifac_size, ifac_key, device=None):
    """Transport.inbound's IFAC step up to the signature check: per packet
    (ifac, unmasked packet) or None where the reference drops it first."""
    n = len(raws)
    if n == 0:
        return []
    buf, off, lens = _pack(raws)
    out_off = off.copy()
    key = np.frombuffer(bytes(ifac_key), np.uint8)
    with _Dev(device) as d:
        p_out = d.alloc(max(int(lens.sum()), 1))
        p_ifac = d.alloc(n * ifac_size)
        p_st = d.alloc(4 * n)
        _native.check(d.lib.rt_ifac_unmask(d.ctx, d.up(buf), d.up(off), d.up(lens), ifac_size, d.up(key), len(key),
                                           p_ifac, p_out, d.up(out_off), p_st, None, n, None))
        st = d.down(p_st, np.zeros(n, np.int32))
        ifac = d.down(p_ifac, np.zeros(n * ifac_size, np.uint8)).tobytes()
        out = d.down(p_out, np.zeros(max(int(lens.sum()), 1), np.uint8)).tobytes()
    res = []
    for i in range(n):
        if st[i] != 0:
            res.append(None)
        else:
            o = int(out_off[i])
            res.append((ifac[i * ifac_size:(i + 1) * ifac_size], out[o:o + int(lens[i]) - ifac_size]))
    return res


# ---------------------------------------------------------------- packets --

def unpack_batch(raws, device=None):
    """Packet.unpack + get_hash over many raw packets: a dict per packet (the
    fields Packet.unpack sets, plus data and packet_hash) or None where
    unpack returns False."""
    n = len(raws)
    if n == 0:
        return []
    buf, off, lens = _pack(raws)
    with _Dev(device) as d:
        p_f = d.alloc(96 * n)
        _native.check(d.lib.rt_packet_unpack(d.ctx, d.up(buf), d.up(off), d.up(lens), p_f, n, None))
        f = d.down(p_f, np.zeros(n, FIELDS_DTYPE))
    res = []
    for i, raw in enumerate(raws):
        r = f[i]
        if not r["ok"]:
            res.append(None)
            continue
        ht = int(r["header_type"])
        do, dl = int(r["data_offset"]), int(r["data_len"])
        res.append({"flags": int(r["flags"]), "hops": int(r["hops"]), "header_type": ht,
                    "context_flag": int(r["context_flag"]), "transport_type": int(r["transport_type"]),
                    "destination_type": int(r["destination_type"]), "packet_type": int(r["packet_type"]),
                    "transport_id": bytes(r["transport_id"]) if ht == 1 else None,
                    "destination_hash": bytes(r["destination_hash"]), "context": int(r["context"]),
                    "data_offset": do, "data": bytes(raw[do:do + dl]), "packet_hash": bytes(r["packet_hash"])})
    return res


def pack_headers_batch(flags, hops, destination_hashes, contexts, transport_ids=None, device=None):
    """Packet.pack's header bytes for many packets (HEADER_2 for all when
    transport_ids is given): returns a list of 19- or 35-byte headers."""
    n = len(flags)
    if n == 0:
        return []
    hl = 35 if transport_ids is not None else 19
    out_off = np.arange(n, dtype=np.uint64) * hl
    with _Dev(device) as d:
        p_out = d.alloc(n * hl)
        _native.check(d.lib.rt_packet_pack_headers(
            d.ctx, d.up(np.asarray(flags, np.uint8)), d.up(np.asarray(hops, np.uint8)),
            None if transport_ids is None else d.up(np.frombuffer(b"".join(transport_ids), np.uint8)),
            d.up(np.frombuffer(b"".join(destination_hashes), np.uint8)), d.up(np.asarray(contexts, np.uint8)),
            p_out, d.up(out_off), n, None))
        out = d.down(p_out, np.zeros(n * hl, np.uint8)).tobytes()
    return [out[i * hl:(i + 1) * hl] for i in range(n)]
