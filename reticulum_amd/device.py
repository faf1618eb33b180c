"""Device-resident batch calls over torch tensors (the measured hot path).

Thin wrappers over rt_encrypt* / rt_decrypt* (include/rnstok.h): every
buffer is a CUDA(HIP) tensor already resident in HBM, the kernels are
enqueued on the given stream (default: torch's current stream) and nothing is
synchronised.  torch is used only for device memory and streams.
"""
import threading

import torch

from . import _native
from .token import KeySet, token_len


def _p(t):
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError("device API needs tensors in device memory")
    if not t.is_contiguous():
        raise ValueError("device API needs contiguous tensors")
    return t.data_ptr()


def _p_rows(t):
    """A (n, row) byte matrix whose rows may sit at any stride >= row (a row
    view of a wider buffer, e.g. 128-B-aligned token rows): bytes within a
    row contiguous; the row stride is passed to the library separately."""
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError("device API needs tensors in device memory")
    if t.dim() != 2 or (t.shape[1] > 1 and t.stride(1) != 1) or (t.shape[0] > 1 and t.stride(0) < t.shape[1]):
        raise ValueError("expected an (n, row) matrix with contiguous rows")
    return t.data_ptr()


def _p_salt(t):
    """Salt rows: contiguous (n, S), or one row broadcast to n
    (`salt[:1].expand(n, S)`, row stride 0: a batch to one identity)."""
    if t is not None and t.dim() == 2 and t.shape[0] > 1 and t.stride(0) == 0 and \
            (t.shape[1] <= 1 or t.stride(1) == 1) and t.is_cuda:
        return t.data_ptr()
    return _p(t)


def _stream(stream, device=None):
    """The HIP stream handle to launch on: ``stream``, else the current
    stream of ``device`` (the tensors' GPU, not whichever GPU is current)."""
    s = stream if stream is not None else torch.cuda.current_stream(device)
    if device is not None and s.device != torch.device(device):
        raise ValueError(f"stream is on {s.device}, the tensors on {device}")
    return s.cuda_stream


def _order_after_current(stream, *tensors):
    """A launch on a side ``stream`` that reads ``tensors`` made on the
    current stream (e.g. a key table an RCCL broadcast just filled; torch only
    makes the *current* stream wait for a collective): the side stream waits
    for the current stream first, and the tensors' memory is kept from reuse
    until the side stream is done with it (the caller may drop them at once)."""
    if stream is None:
        return
    dev = tensors[0].device
    cur = torch.cuda.current_stream(dev)
    if stream == cur:
        return
    stream.wait_stream(cur)
    for t in tensors:
        if t is not None:
            t.record_stream(stream)


def _check_u8(*ts):
    for t in ts:
        if t is not None and t.dtype != torch.uint8:
            raise ValueError("byte buffers must be torch.uint8")


def _check_i32(n, **ts):
    """(n,) contiguous int32 device tensors (None allowed): lengths, statuses
    and key indices are read and written as 32-bit words by the kernels."""
    for name, t in ts.items():
        if t is None:
            continue
        if t.dtype != torch.int32 or t.numel() != n or not t.is_contiguous():
            raise ValueError(f"{name} must be a contiguous ({n},) int32 tensor")


def _check_i64(n, **ts):
    for name, t in ts.items():
        if t is not None and (t.dtype != torch.int64 or t.numel() != n or not t.is_contiguous()):
            raise ValueError(f"{name} must be a contiguous ({n},) int64 tensor")


def _check_rows(name, t, n, width):
    """An (n, row) uint8 matrix whose rows hold at least `width` bytes."""
    if t.dim() != 2 or t.shape[0] != n:
        raise ValueError(f"{name} must be an ({n}, row) uint8 matrix")
    if t.shape[1] < width:
        raise ValueError(f"{name} rows hold {t.shape[1]} bytes, need {width}")


def _check_iv(iv, n):
    if iv.numel() < 16 * n or (iv.dim() == 2 and iv.shape[1] != 16) or not iv.is_contiguous():
        raise ValueError(f"iv must be a contiguous ({n}, 16) uint8 tensor")


def encrypt_uniform(ks: KeySet, pt, pt_len, iv, tok, key_idx=None, stream=None):
    """pt: (n, >= pt_len) uint8 rows; iv: (n, 16) uint8; tok: (n, >=
    token_len(pt_len)) uint8 rows; key_idx: (n,) int32 or None.  pt and tok
    may be row views of wider buffers (their row stride is used)."""
    _check_u8(pt, iv, tok)
    n = pt.shape[0]
    _check_rows("pt", pt, n, pt_len)
    _check_rows("tok", tok, n, token_len(pt_len))
    _check_iv(iv, n)
    _check_i32(n, key_idx=key_idx)
    lib = _native.load()
    _native.check(lib.rt_encrypt_uniform(ks.handle, _p_rows(pt), pt.stride(0), pt_len, _p(key_idx), _p(iv),
                                         _p_rows(tok), tok.stride(0), n, _stream(stream, pt.device)))


def decrypt_uniform(ks: KeySet, tok, tok_len, pt, out_len, status, key_idx=None, stream=None):
    """tok: (n, >= tok_len) uint8 holding tok_len-byte tokens; pt: (n, >=
    tok_len - 48) uint8; out_len/status/key_idx: (n,) int32."""
    _check_u8(tok, pt)
    n = tok.shape[0]
    _check_rows("tok", tok, n, tok_len)
    _check_rows("pt", pt, n, max(tok_len - 48, 0))
    _check_i32(n, out_len=out_len, status=status, key_idx=key_idx)
    lib = _native.load()
    _native.check(lib.rt_decrypt_uniform(ks.handle, _p_rows(tok), tok.stride(0), tok_len, _p(key_idx), _p_rows(pt),
                                         pt.stride(0), _p(out_len), _p(status), n, _stream(stream, tok.device)))


# ------------------------------------------------- unit-interleaved layout --
# For batches that live on the device from end to end (rt_encrypt_interleaved,
# include/rnstok.h): 16-B unit u of packet p at 16*(u*n + p), i.e. a (U, n, 16)
# uint8 tensor, so every wave load/store is one contiguous KiB of HBM.

def units(nbytes):
    """16-B units that hold nbytes."""
    return (int(nbytes) + 15) // 16


def interleave(rows, nbytes=None):
    """(n, >= nbytes) uint8 rows -> the (units(nbytes), n, 16) interleaved
    tensor (a copy; the last unit zero-padded)."""
    n = rows.shape[0]
    L = rows.shape[1] if nbytes is None else int(nbytes)
    U = units(L)
    out = torch.zeros((n, U * 16), dtype=torch.uint8, device=rows.device)
    out[:, :L] = rows[:, :L]
    return out.view(n, U, 16).transpose(0, 1).contiguous()


def deinterleave(u, nbytes=None):
    """(U, n, 16) interleaved units -> (n, nbytes) rows (a copy)."""
    U, n, _ = u.shape
    rows = u.transpose(0, 1).reshape(n, U * 16)
    return rows[:, : (U * 16 if nbytes is None else int(nbytes))].contiguous()


# ---- rows in 128-B-aligned slots ------
LINE = 128


def aligned_rows(n, width, phase=0, device=None):
    """An (n, width) uint8 row view for the uniform entry points whose row
    stride is a multiple of 128 B and whose byte ``phase`` of every row starts
    a 128-B line: phase 0 for plaintexts, 16 for tokens (the ciphertext after
    the IV), 35 for HEADER_1 packets.  Same outputs as packed rows; the chip
    runs the token kernels 3-5 % faster on them (fewer lines straddle two
    packets).  The bytes between rows are uninitialised."""
    n, width, phase = int(n), int(width), int(phase)
    if n < 0 or width < 0 or not 0 <= phase < LINE:
        raise ValueError("aligned_rows: n, width >= 0 and 0 <= phase < 128")
    stride = max(LINE, -(-width // LINE) * LINE)
    buf = torch.empty(n * stride + LINE, dtype=torch.uint8, device=device)
    off = (-(buf.data_ptr() + phase)) % LINE
    return buf[off:off + n * stride].view(n, stride)[:, :width] if n else buf[:0].view(0, width)


def _check_units(name, t, U, n):
    if t.dtype != torch.uint8 or t.dim() != 3 or tuple(t.shape) != (U, n, 16) or not t.is_contiguous():
        raise ValueError(f"{name} must be a contiguous ({U}, {n}, 16) uint8 tensor of interleaved units")


def encrypt_interleaved(ks: KeySet, pt, pt_len, iv, tok, key_idx=None, stream=None):
    """Token.encrypt of n packets of pt_len bytes in the interleaved layout:
    pt (units(pt_len), n, 16), iv (n, 16), tok (token_len(pt_len)/16, n, 16).
    Tokens are bit-identical to encrypt_uniform's."""
    n = iv.shape[0]
    _check_units("pt", pt, units(pt_len), n)
    _check_units("tok", tok, token_len(pt_len) // 16, n)
    _check_u8(iv)
    _check_iv(iv, n)
    _check_i32(n, key_idx=key_idx)
    lib = _native.load()
    _native.check(lib.rt_encrypt_interleaved(ks.handle, _p(pt) if pt.numel() else None, pt_len, _p(key_idx), _p(iv),
                                             _p(tok), n, _stream(stream, tok.device)))


def decrypt_interleaved(ks: KeySet, tok, tok_len, pt, out_len, status, key_idx=None, stream=None):
    """Token.decrypt of n tokens of tok_len = 48 + 16k bytes (k >= 1) in the
    interleaved layout: tok (tok_len/16, n, 16), pt ((tok_len-48)/16, n, 16)
    (plaintext incl. its pad block, zeroed on failure), out_len/status (n,)
    int32 as decrypt_uniform."""
    n = tok.shape[1] if tok.dim() == 3 else -1
    if tok_len < 64 or tok_len % 16:
        raise ValueError("interleaved tokens must be 48 + 16*k bytes, k >= 1")
    _check_units("tok", tok, tok_len // 16, n)
    _check_units("pt", pt, (tok_len - 48) // 16, n)
    _check_i32(n, out_len=out_len, status=status, key_idx=key_idx)
    lib = _native.load()
    _native.check(lib.rt_decrypt_interleaved(ks.handle, _p(tok), tok_len, _p(key_idx), _p(pt), _p(out_len),
                                             _p(status), n, _stream(stream, tok.device)))


def verify(ks: KeySet, tok, tok_off, tok_len, status, key_idx=None, stream=None):
    """Token.verify_hmac (Token.py:77-84) over device buffers, no AES: token
    i is tok[tok_off[i] : +tok_len[i]] (int64 / int32); status (n,) int32
    receives RT_ST_OK (tag valid), RT_ST_BAD_HMAC or RT_ST_TOO_SHORT."""
    _check_u8(tok)
    n = tok_off.numel()
    _check_i64(n, tok_off=tok_off)
    _check_i32(n, tok_len=tok_len, status=status, key_idx=key_idx)
    lib = _native.load()
    _native.check(lib.rt_verify(ks.handle, _p(tok), _p(tok_off), _p(tok_len), _p(key_idx), _p(status), n,
                                _stream(stream, tok.device)))


def verify_trials(ks: KeySet, tok, tok_off, tok_len, pair_off, pair_key, first, stream=None):
    """Ratchet trials (Identity.py:865-878) over device buffers: token t is
    tok[tok_off[t] : +tok_len[t]] (int64 / int32), its candidates are
    pair_key[pair_off[t] : pair_off[t+1]] (int32, pair_off (n+1,) int32 from
    0); first (n,) int32 receives the rank of the first candidate whose key
    opens token t, or -1."""
    _check_u8(tok)
    n = tok_off.numel()
    _check_i64(n, tok_off=tok_off)
    _check_i32(n, tok_len=tok_len, first=first)
    _check_i32(n + 1, pair_off=pair_off)
    _check_i32(pair_key.numel(), pair_key=pair_key)
    lib = _native.load()
    _native.check(lib.rt_verify_trials(ks.handle, _p(tok), _p(tok_off), _p(tok_len), _p(pair_off), _p(pair_key),
                                       _p(first), n, pair_key.numel(), _stream(stream, tok.device)))


def _workspace(n, device):
    lib = _native.load()
    return torch.empty(int(lib.rt_workspace_bytes(n)), dtype=torch.uint8, device=device)


def encrypt(ks: KeySet, pt, pt_off, pt_len, iv, tok, tok_off, key_idx=None, stream=None, sort=False,
            workspace=None):
    """Variable-length batch: pt/tok flat uint8 buffers, pt_off/tok_off int64,
    pt_len int32, iv (n,16) uint8.  ``sort=True`` groups packets by length on
    the device first (same outputs; wavefronts carry similar lengths)."""
    _check_u8(pt, iv, tok)
    n = pt_off.numel()
    _check_i64(n, pt_off=pt_off, tok_off=tok_off)
    _check_i32(n, pt_len=pt_len, key_idx=key_idx)
    _check_iv(iv, n)
    lib = _native.load()
    if sort:
        ws = workspace if workspace is not None else _workspace(n, pt.device)
        _native.check(lib.rt_encrypt_ex(ks.handle, _p(pt), _p(pt_off), _p(pt_len), _p(key_idx), _p(iv), _p(tok),
                                        _p(tok_off), n, _native.RT_F_SORT_BY_LENGTH, _p(ws), _stream(stream, pt.device)))
        return
    _native.check(lib.rt_encrypt(ks.handle, _p(pt), _p(pt_off), _p(pt_len), _p(key_idx), _p(iv), _p(tok),
                                 _p(tok_off), n, _stream(stream, pt.device)))


def decrypt(ks: KeySet, tok, tok_off, tok_len, pt, pt_off, out_len, status, key_idx=None, stream=None, sort=False,
            workspace=None):
    _check_u8(tok, pt)
    n = tok_off.numel()
    _check_i64(n, tok_off=tok_off, pt_off=pt_off)
    _check_i32(n, tok_len=tok_len, out_len=out_len, status=status, key_idx=key_idx)
    lib = _native.load()
    if sort:
        ws = workspace if workspace is not None else _workspace(n, tok.device)
        _native.check(lib.rt_decrypt_ex(ks.handle, _p(tok), _p(tok_off), _p(tok_len), _p(key_idx), _p(pt),
                                        _p(pt_off), _p(out_len), _p(status), n, _native.RT_F_SORT_BY_LENGTH, _p(ws),
                                        _stream(stream, tok.device)))
        return
    _native.check(lib.rt_decrypt(ks.handle, _p(tok), _p(tok_off), _p(tok_len), _p(key_idx), _p(pt), _p(pt_off),
                                 _p(out_len), _p(status), n, _stream(stream, tok.device)))


def hkdf(ikm, out, salt=None, context=None, stream=None):
    """HKDF-SHA256 over device rows (RNS/Cryptography/HKDF.py:35-62): ikm
    (n, L) uint8, salt (n, S) uint8 or None (the reference's 32 zero bytes;
    one row expanded to (n, S) is shared, its HMAC midstates computed once),
    context a (C,) uint8 device tensor or None, out (n, length) uint8 with
    length = out.shape[1] >= 1.  Row i of out = hkdf(length, ikm[i], salt[i],
    context)."""
    _check_u8(ikm, out, salt, context)
    n = ikm.shape[0]
    if out.shape[0] != n or (salt is not None and salt.shape[0] != n):
        raise ValueError("shape mismatch")
    length = out.shape[1]
    lib = _native.load()
    ctx = _native.context(out.device.index)
    _native.check(lib.rt_hkdf(ctx, _p(ikm), ikm.stride(0), ikm.shape[1], _p_salt(salt),
                              salt.stride(0) if salt is not None else 0, salt.shape[1] if salt is not None else 0,
                              _p(context), context.numel() if context is not None else 0, _p(out), out.stride(0),
                              length, n, _stream(stream, ikm.device)))


def keyset(keys, stream=None):
    """KeySet from a device key table (Token.py:58-74 per row): ``keys`` is a
    contiguous (n_keys, 64 or 32) uint8 CUDA tensor, e.g. received by
    shard.broadcast_keys; expanded on its device on ``stream`` without a
    host round trip.  Usable from any stream right away, as derive_keyset."""
    _check_u8(keys)
    if keys.dim() != 2 or keys.shape[1] not in (32, 64) or keys.shape[0] < 1 or not keys.is_contiguous():
        raise ValueError("keys must be a contiguous (n_keys, 64 or 32) uint8 device tensor")
    n, klen = keys.shape
    lib = _native.load()
    ctx = _native.context(keys.device.index)
    _order_after_current(stream, keys)
    h = lib.rt_keyset_create_device(ctx, _p(keys), klen, n, _stream(stream, keys.device))
    if not h:
        raise _native.NativeError(-1, _native.last_error())
    return KeySet._adopt(h, klen, n, lib, ctx)


def derive_keyset(ikm, salt=None, context=None, key_len=64, stream=None):
    """Per-packet keying from device rows (Identity.py:837-846): KeySet whose
    key i is Token(hkdf(key_len, ikm[i], salt[i], context)); derived and
    expanded on the device in one launch (the derived keys never reach HBM)
    on ``stream``.  The key set is usable from any stream or host call right
    away: every later launch that reads it waits for this build first."""
    _check_u8(ikm, salt, context)
    n = ikm.shape[0]
    lib = _native.load()
    ctx = _native.context(ikm.device.index)
    _order_after_current(stream, ikm, salt, context)
    h = lib.rt_keyset_create_hkdf(ctx, _p(ikm), ikm.stride(0), ikm.shape[1], _p_salt(salt),
                                  salt.stride(0) if salt is not None else 0, salt.shape[1] if salt is not None else 0,
                                  _p(context), context.numel() if context is not None else 0, key_len, n,
                                  _stream(stream, ikm.device))
    if not h:
        raise _native.NativeError(-1, _native.last_error())
    return KeySet._adopt(h, key_len, n, lib, ctx)


def map_hashes(data, out, salts, part_off=None, part_len=None, part_res=None, sdu=464, guard=0,
               first_collision=None, stream=None):
    """Resource map hashes over device buffers (Resource.py:505-506): out
    (n_parts*4,) uint8; salts (n_res, S) uint8 (random hashes); with
    part_off (int64) / part_len (int32) the parts are arbitrary slices of
    ``data`` and part_res (int32) names each part's resource, otherwise
    ``data`` is one resource cut into ``sdu``-byte parts.  first_collision
    (n_res,) int32 receives the first part index repeating a map hash of the
    previous ``guard`` parts, or -1."""
    _check_u8(data, out, salts)
    n_parts = out.numel() // 4
    lib = _native.load()
    ctx = _native.context(data.device.index)
    _native.check(lib.rt_map_hashes(ctx, _p(data), _p(part_off), _p(part_len), data.numel(), sdu, _p(salts),
                                    salts.shape[1], _p(part_res), salts.shape[0], guard, _p(out),
                                    _p(first_collision), n_parts, _stream(stream, data.device)))


# ---------------------------------------------------------------- wire side --
# Device-resident forms of reticulum_amd.wire (wire_kernels.hip): flat uint8
# buffers, int64 offsets, int32 lengths, enqueued on the stream, no sync.

def _ctx_of(t):
    return _native.context(t.device.index)


def hdlc_frame(pkt, pkt_off, pkt_len, out, frame_off, workspace=None, stream=None):
    """HDLC framing (TCPInterface.py:44-53, 323) of n packets into ``out`` in
    order: frame i = 7E || escape(packet i) || 7E at out[frame_off[i]:
    frame_off[i+1]]; frame_off (n+1,) int64, frame_off[n] = total bytes; out
    needs sum(2*len+2) bytes at most."""
    _check_u8(pkt, out)
    n = pkt_off.numel()
    if pkt_len.numel() != n or frame_off.numel() != n + 1:
        raise ValueError("shape mismatch")
    lib = _native.load()
    ws = workspace if workspace is not None else torch.empty(
        int(lib.rt_hdlc_frame_workspace_bytes(n)), dtype=torch.uint8, device=pkt.device)
    _native.check(lib.rt_hdlc_frame(_ctx_of(pkt), _p(pkt), _p(pkt_off), _p(pkt_len), n, _p(out), _p(frame_off),
                                    _p(ws), _stream(stream, pkt.device)))


def deframe_slots_bytes(nbytes, max_pairs):
    """Output capacity hdlc_deframe needs with ``line_phase`` (slots)."""
    return int(nbytes) + LINE * (int(max_pairs) + 1)


def hdlc_deframe(buf, out, frame_off, frame_len, status, counts, hw_mtu=262144, ifac_size=0, workspace=None,
                 stream=None, line_phase=None):
    """One pass of the HDLC read loop (TCPInterface.py:387-410) over ``buf``:
    for each consecutive flag pair k (at most frame_off.numel() pairs) the
    unescaped frame at out[frame_off[k]: frame_off[k] + frame_len[k]] with its
    RT_FRAME_* status; counts (2,) int64 = [pairs, bytes consumed].  With
    ``line_phase`` (0..127) each frame gets a 128-B-aligned slot whose byte
    line_phase starts a line (rt_hdlc_deframe_slots; ``out`` then needs
    deframe_slots_bytes(len(buf), max_pairs) bytes), else it sits at its
    position in buf."""
    _check_u8(buf, out)
    max_pairs = frame_off.numel()
    need = buf.numel() if line_phase is None else deframe_slots_bytes(buf.numel(), max_pairs)
    if frame_len.numel() != max_pairs or status.numel() != max_pairs or counts.numel() < 2 or out.numel() < need:
        raise ValueError("shape mismatch")
    lib = _native.load()
    ws = workspace if workspace is not None else torch.empty(
        int(lib.rt_hdlc_deframe_workspace_bytes(buf.numel())), dtype=torch.uint8, device=buf.device)
    if line_phase is None:
        _native.check(lib.rt_hdlc_deframe(_ctx_of(buf), _p(buf), buf.numel(), hw_mtu, ifac_size, _p(out),
                                          _p(frame_off), _p(frame_len), _p(status), _p(counts), max_pairs, _p(ws),
                                          _stream(stream, buf.device)))
    else:
        _native.check(lib.rt_hdlc_deframe_slots(_ctx_of(buf), _p(buf), buf.numel(), hw_mtu, ifac_size, int(line_phase),
                                                _p(out), _p(frame_off), _p(frame_len), _p(status), _p(counts),
                                                max_pairs, _p(ws), _stream(stream, buf.device)))


def frames_compact(frame_off, frame_len, status, counts, f_off, f_len, frame_pair, n_frames, workspace=None,
                   stream=None):
    """The frames an hdlc_deframe pass hands on (pair k < counts[0] with
    status RT_FRAME_OK; TCPInterface.py:391-401), in stream order, to the
    front of f_off (int64) / f_len (int32) / frame_pair (int64, the pair
    index); n_frames (a 0-d int64 device tensor) gets their number, and the
    entries past it are f_off 0, f_len 0, frame_pair -1.  All arrays have
    max_pairs = frame_off.numel() entries."""
    max_pairs = frame_off.numel()
    if any(t.numel() != max_pairs for t in (frame_len, status, f_off, f_len, frame_pair)) or \
            counts.numel() < 2 or n_frames.numel() != 1:
        raise ValueError("shape mismatch")
    if frame_off.dtype != torch.int64 or f_off.dtype != torch.int64 or frame_pair.dtype != torch.int64 or \
            n_frames.dtype != torch.int64 or frame_len.dtype != torch.int32 or f_len.dtype != torch.int32 or \
            status.dtype != torch.int32 or counts.dtype != torch.int64:
        raise TypeError("frames_compact: int64 offsets/pairs/counts, int32 lengths/status")
    lib = _native.load()
    ws = workspace if workspace is not None else torch.empty(
        max(1, int(lib.rt_frames_compact_workspace_bytes(max_pairs))), dtype=torch.uint8, device=frame_off.device)
    _native.check(lib.rt_frames_compact(_ctx_of(frame_off), _p(frame_off), _p(frame_len), _p(status), _p(counts),
                                        max_pairs, _p(f_off), _p(f_len), _p(frame_pair), _p(n_frames), _p(ws),
                                        _stream(stream, frame_off.device)))


def token_spans(fields, pkt_off, tok_off, tok_len, stream=None):
    """Packet.unpack's data (Packet.py:262-275), the token of each packet:
    tok_off[i] = pkt_off[i] + data_offset, tok_len[i] = data_len where
    fields[i] (an rt_packet_fields record from packet_unpack) is ok, else
    pkt_off[i] and 0.  int64 offsets, int32 lengths."""
    n = pkt_off.numel()
    if fields.numel() != 96 * n or tok_off.numel() != n or tok_len.numel() != n:
        raise ValueError("shape mismatch")
    if pkt_off.dtype != torch.int64 or tok_off.dtype != torch.int64 or tok_len.dtype != torch.int32:
        raise TypeError("token_spans: int64 offsets, int32 lengths")
    lib = _native.load()
    _native.check(lib.rt_token_spans(_ctx_of(fields), _p(fields), _p(pkt_off), n, _p(tok_off), _p(tok_len),
                                     _stream(stream, fields.device)))


def ifac_mask(pkt, pkt_off, pkt_len, ifac, ifac_key, out, out_off, stream=None):
    """Transport.transmit's IFAC step (Transport.py:1069-1101): packet i plus
    its access code ifac[i] (n, ifac_size) -> pkt_len[i] + ifac_size masked
    bytes at out[out_off[i]:]; ifac_key (K,) uint8, K <= 64."""
    _check_u8(pkt, ifac, ifac_key, out)
    n = pkt_off.numel()
    if pkt_len.numel() != n or ifac.shape[0] != n or out_off.numel() != n:
        raise ValueError("shape mismatch")
    lib = _native.load()
    _native.check(lib.rt_ifac_mask(_ctx_of(pkt), _p(pkt), _p(pkt_off), _p(pkt_len), _p(ifac), ifac.shape[1],
                                   _p(ifac_key), ifac_key.numel(), _p(out), _p(out_off), n, _stream(stream, pkt.device)))


def ifac_unmask(pkt, pkt_off, pkt_len, ifac_key, ifac_out, out, out_off, status, out_len=None, stream=None):
    """Transport.inbound's IFAC step up to the signature check
    (Transport.py:1441-1475): status[i] = 0 with the IFAC in ifac_out[i] (n,
    ifac_size) and the unmasked packet (pkt_len[i] - ifac_size bytes) at
    out[out_off[i]:], or 1 where the reference drops the packet first.
    out_len (n,) int32, if given, receives pkt_len[i] - ifac_size where the
    status is 0 and 0 elsewhere (packet_unpack's lengths)."""
    _check_u8(pkt, ifac_key, ifac_out, out)
    n = pkt_off.numel()
    if pkt_len.numel() != n or ifac_out.shape[0] != n or out_off.numel() != n or status.numel() != n or \
            (out_len is not None and (out_len.numel() != n or out_len.dtype != torch.int32)):
        raise ValueError("shape mismatch")
    lib = _native.load()
    _native.check(lib.rt_ifac_unmask(_ctx_of(pkt), _p(pkt), _p(pkt_off), _p(pkt_len), ifac_out.shape[1],
                                     _p(ifac_key), ifac_key.numel(), _p(ifac_out), _p(out), _p(out_off), _p(status),
                                     _p(out_len), n, _stream(stream, pkt.device)))


def packet_unpack(pkt, pkt_off, pkt_len, fields, stream=None):
    """Packet.unpack + get_hash (Packet.py:242-275, 342-353): fields (n, 96)
    uint8 receives one rt_packet_fields record per packet
    (reticulum_amd.wire.FIELDS_DTYPE)."""
    _check_u8(pkt, fields)
    n = pkt_off.numel()
    if pkt_len.numel() != n or fields.numel() != 96 * n:
        raise ValueError("shape mismatch")
    lib = _native.load()
    _native.check(lib.rt_packet_unpack(_ctx_of(pkt), _p(pkt), _p(pkt_off), _p(pkt_len), _p(fields), n,
                                       _stream(stream, pkt.device)))


def pack_headers(flags, hops, destination_hash, context, out, out_off, transport_id=None, stream=None):
    """Packet.pack's header (Packet.py:167-228) for n packets at
    out[out_off[i]:]: flags, hops, [transport_id], destination hash, context
    (19 or 35 bytes).  flags/hops/context (n,) uint8; hashes (n, 16) uint8."""
    _check_u8(flags, hops, destination_hash, context, out, transport_id)
    n = flags.numel()
    lib = _native.load()
    _native.check(lib.rt_packet_pack_headers(_ctx_of(out), _p(flags), _p(hops), _p(transport_id),
                                             _p(destination_hash), _p(context), _p(out), _p(out_off), n,
                                             _stream(stream, out.device)))


# ------------------------------------------------------- host-origin path --

def copy_to_host(dst, src, stream=None):
    """Enqueue ``dst.copy_(src)`` for a device tensor ``src`` and a host tensor
    ``dst`` of the same size, both contiguous, through rt_memcpy_d2h: a pinned
    ``dst`` is written by GPU stores into the mapped host buffer
    (copy_kernels.hip; 54 GB/s alone and 87 GB/s beside a copy-engine H2D on
    MI355X, against 30 GB/s for the copy engine's D2H,
    profiles/r03n_pcie_probe.json), a pageable one by hipMemcpyAsync.  Like
    ``copy_(non_blocking=True)`` nothing is synchronised: ``dst`` is valid
    once ``stream`` (default: the current stream of src's GPU) has run."""
    if not src.is_cuda or dst.is_cuda:
        raise ValueError("copy_to_host copies a device tensor into a host tensor")
    if not src.is_contiguous() or not dst.is_contiguous():
        raise ValueError("copy_to_host needs contiguous tensors")
    nbytes = src.numel() * src.element_size()
    if dst.numel() * dst.element_size() != nbytes:
        raise ValueError("copy_to_host: size mismatch")
    if nbytes == 0:
        return
    lib = _native.load()
    _native.check(lib.rt_memcpy_d2h(_ctx_of(src), dst.data_ptr(), src.data_ptr(), nbytes,
                                    _stream(stream, src.device)))


def copy_to_host_upto(dst, src, nbytes_dev, stream=None):
    """Enqueue the copy of the first min(dst size, nbytes_dev) bytes of the
    device tensor ``src`` into the pinned host tensor ``dst``, where
    ``nbytes_dev`` is a one-element int64 DEVICE tensor read at run time (e.g.
    ``frame_off[n]`` from hdlc_frame: the stream's length, which the host
    does not know without a sync; zero or negative copies nothing) — GPU
    stores into the mapped buffer (rt_memcpy_d2h_upto).  Nothing is
    synchronised; bytes of ``dst`` past the count are left as they were."""
    if not src.is_cuda or dst.is_cuda or not dst.is_pinned():
        raise ValueError("copy_to_host_upto copies a device tensor into a pinned host tensor")
    if not src.is_contiguous() or not dst.is_contiguous():
        raise ValueError("copy_to_host_upto needs contiguous tensors")
    if nbytes_dev.dtype != torch.int64 or nbytes_dev.numel() != 1 or not nbytes_dev.is_cuda:
        raise TypeError("nbytes_dev: one int64 element on the device")
    if nbytes_dev.device != src.device:
        raise ValueError("nbytes_dev must be on src's device")
    nbytes = min(src.numel() * src.element_size(), dst.numel() * dst.element_size())
    if nbytes == 0:
        return
    lib = _native.load()
    _native.check(lib.rt_memcpy_d2h_upto(_ctx_of(src), dst.data_ptr(), src.data_ptr(), nbytes, _p(nbytes_dev),
                                         _stream(stream, src.device)))


# ------------------------------------------------------------ launch clock --

CLOCK_KERNELS = ("encrypt", "decrypt")      # RT_CLOCK_ENCRYPT, RT_CLOCK_DECRYPT
REALTIME_HZ = 100e6                         # s_memrealtime ticks per second


def clock_summary(words):
    """The rt_clock_stamps words (8 ints) as per-kernel figures: the run's
    sustained shader clock (cycles / real-time ticks x 100 MHz), the cycles
    per launch (the mean workgroup span: one persistent workgroup per CU)
    and the mean workgroup span in ms.  Kernels with no stamped launch are
    left out."""
    out = {}
    for k, name in enumerate(CLOCK_KERNELS):
        cyc, ticks, wgs, launches = (int(x) for x in words[4 * k:4 * k + 4])
        if wgs == 0 or ticks == 0:
            continue
        out[name] = {"clock_ghz": cyc / ticks * REALTIME_HZ / 1e9, "cycles_per_launch": cyc / wgs,
                     "wg_span_ms": ticks / wgs / REALTIME_HZ * 1e3, "launches": launches,
                     "workgroups_per_launch": wgs / launches if launches else None}
    return out


class LaunchClock:
    """Stamp every encrypt/decrypt launch of a block on ``device``'s context
    (rt_clock_stamps) and read the run's clock afterwards::

        with device.LaunchClock(dev) as lc:
            ...launches...
        lc.summary()      # syncs the device, then clock_summary(words)

    Stamping is per context, i.e. process-wide for the device: every launch
    on it from any thread or stream while the block is open is stamped into
    this object's words.  One block per device at a time (a nested or
    concurrent block raises RuntimeError instead of mixing stamps), and the
    exit waits for the device, so no launch still adds to the words once the
    block is closed."""

    _open = set()               # device indices with an open block
    _open_lock = threading.Lock()

    def __init__(self, dev=None):
        dev = torch.device("cuda", torch.cuda.current_device()) if dev is None else torch.device(dev)
        self.dev = dev
        self._index = dev.index if dev.index is not None else torch.cuda.current_device()
        self.acc = torch.zeros(8, dtype=torch.int64, device=dev)
        self._ctx = _native.context(self._index)

    def __enter__(self):
        with LaunchClock._open_lock:
            if self._index in LaunchClock._open:
                raise RuntimeError(f"a LaunchClock is already open on cuda:{self._index}: stamping is per context")
            LaunchClock._open.add(self._index)
        try:
            # the zeroed words are ordered before any launch the block enqueues
            torch.cuda.synchronize(self.dev)
            _native.check(_native.load().rt_clock_stamps(self._ctx, self.acc.data_ptr()))
        except BaseException:
            with LaunchClock._open_lock:
                LaunchClock._open.discard(self._index)
            raise
        return self

    def __exit__(self, *exc):
        try:
            _native.check(_native.load().rt_clock_stamps(self._ctx, None))
            # launches already queued still add to acc: let them land before
            # the block counts as closed (and before acc can be freed)
            torch.cuda.synchronize(self.dev)
        finally:
            with LaunchClock._open_lock:
                LaunchClock._open.discard(self._index)
        return False

    def words(self):
        torch.cuda.synchronize(self.dev)
        return [int(x) for x in self.acc.cpu()]

    def summary(self):
        return clock_summary(self.words())
