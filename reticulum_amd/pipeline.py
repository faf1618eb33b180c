"""A Reticulum interface's packet path, device-resident end to end
("what surrounds the token on the interface path ... needed
for a true end-to-end node pipeline").

Outbound, as a node sends DATA packets through an interface with IFAC:
    Token.encrypt            Token.py:87-97 (Packet.pack -> Destination/Link.encrypt)
    Packet.pack header       Packet.py:178-228
    IFAC mask                Transport.py:1069-1101 (transmit)
    HDLC framing             TCPInterface.py:44-53, 323 (process_outgoing)
Inbound, as the interface's read loop hands frames to Transport:
    HDLC deframing           TCPInterface.py:387-410 (read_loop)
    IFAC unmask              Transport.py:1441-1475 (inbound; the Ed25519
                             signature check that follows, :1477-1481, stays
                             with the caller: `ifac` is returned for it)
    Packet.unpack + hash     Packet.py:242-275, 342-353
    Token.decrypt            Token.py:100-114 (Link/Identity.decrypt)

Every stage is one of reticulum_amd.device's kernels, the rearranging of
offsets and lengths between them included (frames_compact, token_spans), and
nothing is synchronised: sizes the host does not know (the number of frames
in a stream) stay on the device, and entries past them carry length 0, which
every later stage rejects like the reference does (a frame too short for its
IFAC, a packet too short for its header, a token too short for its tag).
With ``stream`` given, every launch and every temporary is on that stream
(allocated there, so the caching allocator never hands a temporary to other
work before the stream is done with it) and so are the results: the caller
makes its own stream wait on it before reading them.
"""
import contextlib

import torch

from . import device
from .token import KeySet, token_len

HEADER_1_LEN = 19           # flags, hops, destination hash (16), context: Packet.py:178-228
FRAME_OK = 0                # RT_FRAME_OK (include/rnstok.h)
# Outbound builds its packets in 128-B-aligned slots with each HEADER_1
# packet's token ciphertext (packet + 19 + 16 B of IV) starting on a line: the
# token encrypt and the IFAC mask then fetch fewer lines twice (DESIGN.md §3,
# "Rows in 128-B-aligned slots"; §4.8).
CT_PHASE = HEADER_1_LEN + 16


def outbound(ks: KeySet, pt, iv, destination_hash, context, ifac, ifac_key, flags=None, hops=None, stream=None,
             aligned=True):
    """n DATA packets of one length L, one link key: pt (n, L) uint8, iv (n,
    16), destination_hash (n, 16), context (n,) uint8, flags/hops (n,) uint8
    (default 0: HEADER_1 DATA, hop 0), ifac (n, ifac_size) the access codes
    (the tail of the interface identity's signature of each packet, made by
    the caller; None or zero columns: an interface without IFAC, no mask),
    ifac_key (K,) uint8 (unused without IFAC).  Returns (stream, frame_off): the HDLC
    byte stream is stream[:frame_off[n]] (int64 on the device), frame i at
    stream[frame_off[i]:frame_off[i+1]].  ``aligned`` (default) builds the
    packets in 128-B-aligned slots (token ciphertext on a line); False packs
    them end to end.  The stream is the same either way."""
    with _on(stream):      # temporaries allocated on the stream that uses them
        n, L = pt.shape
        dev = pt.device
        flags = flags if flags is not None else torch.zeros(n, dtype=torch.uint8, device=dev)
        hops = hops if hops is not None else torch.zeros(n, dtype=torch.uint8, device=dev)
        pl = HEADER_1_LEN + token_len(L)
        isz = ifac.shape[1] if ifac is not None else 0
        if aligned:
            raw = device.aligned_rows(n, pl, CT_PHASE, dev)
            stride = raw.stride(0)
            flat = raw.as_strided((n * stride,), (1,))
        else:
            stride = pl
            flat = torch.empty(n * stride, dtype=torch.uint8, device=dev)
            raw = flat.view(n, pl)
        device.encrypt_uniform(ks, pt, L, iv, raw[:, HEADER_1_LEN:], stream=stream)
        off = torch.arange(n, dtype=torch.int64, device=dev) * stride
        device.pack_headers(flags, hops, destination_hash, context, flat, off, stream=stream)
        if isz:
            ml = pl + isz
            masked = torch.empty(n * ml, dtype=torch.uint8, device=dev)
            m_off = torch.arange(n, dtype=torch.int64, device=dev) * ml
            device.ifac_mask(flat, off, torch.full((n,), pl, dtype=torch.int32, device=dev), ifac, ifac_key, masked,
                             m_off, stream=stream)
        else:
            # an interface without IFAC transmits the packet as packed
            # (Transport.py:1069-1071: the mask applies only with ifac_identity)
            ml, masked, m_off = pl, flat, off
        framed = torch.empty(n * (2 * ml + 2), dtype=torch.uint8, device=dev)
        frame_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        device.hdlc_frame(masked, m_off, torch.full((n,), ml, dtype=torch.int32, device=dev), framed, frame_off,
                          stream=stream)
    return framed, frame_off


def inbound(ks: KeySet, buf, ifac_key, ifac_size, max_pairs, hw_mtu=262144, stream=None, aligned=None):
    """One read of an interface's byte stream ``buf`` (uint8 on the device)
    through deframing, IFAC unmask (skipped for ``ifac_size`` 0, an interface
    without access codes: then frames with the IFAC flag set are dropped, as
    Transport.py:1482-1486 does), unpack and token decrypt, for at most
    ``max_pairs`` consecutive flag pairs (a stream of n frames has 2n - 1:
    frames and the empty gaps between them).

    Returns a dict of device tensors.  Per flag pair k: ``frame_status``
    (RT_FRAME_*; -1 past the pairs found), ``frame_len`` (its unescaped
    length) and ``counts`` = [pairs, bytes
    consumed] as the read loop leaves them (TCPInterface.py:391-411).  The
    frames the read loop hands on (RT_FRAME_OK) are compacted in stream order
    into the first ``n_frames`` (a device scalar) entries of the per-frame
    arrays, whose remaining entries are empty: ``frame_pair`` (their pair
    index), ``ifac_status`` (0: unmasked; 1: dropped before the signature
    check), ``ifac`` (the access code for the caller's signature check),
    ``fields`` (rt_packet_fields; ok = 0 where unpack fails), and the token's
    outcome: ``status`` (RT_* token status; TOO_SHORT where there is no
    packet) with the plaintext at ``pt[pt_off[i]: pt_off[i] + pt_len[i]]``.
    Compacting first keeps the per-packet kernels' waves full (the gaps
    between frames would otherwise be half of every wave).  With ``aligned``
    the deframer writes every frame into its own 128-B-aligned slot
    (rt_hdlc_deframe_slots: a HEADER_1 packet's token ciphertext on a line,
    128 B more buffer per pair of max_pairs), the unmasked packets stay at
    those offsets and each plaintext starts on a line too; otherwise frames
    sit at their stream offsets.  Only the offsets differ (DESIGN.md §4.8:
    −8 % for the path, mostly the unmask reading slotted frames).  The default
    (None) takes slots when their padding is at most the stream's own size
    (a Reticulum stream has about two pairs per packet; a max_pairs sized for
    a stream of nothing but flags would multiply the buffers instead)."""
    if aligned is None:
        aligned = device.LINE * (max_pairs + 1) <= buf.numel()
    with _on(stream):      # temporaries allocated on the stream that uses them
        dev = buf.device
        # (at least one byte: an empty read still gives every later stage a
        # buffer to point at; no frame ever reaches into it)
        nout = device.deframe_slots_bytes(buf.numel(), max_pairs) if aligned else buf.numel()
        out = torch.empty(max(nout, 1), dtype=torch.uint8, device=dev)
        d_off = torch.empty(max_pairs, dtype=torch.int64, device=dev)
        d_len = torch.empty(max_pairs, dtype=torch.int32, device=dev)
        d_st = torch.full((max_pairs,), -1, dtype=torch.int32, device=dev)
        counts = torch.empty(2, dtype=torch.int64, device=dev)
        device.hdlc_deframe(buf, out, d_off, d_len, d_st, counts, hw_mtu=hw_mtu, ifac_size=ifac_size, stream=stream,
                            line_phase=CT_PHASE if aligned else None)
        # the frames handed on, to the front in stream order; empty entries past them
        f_off = torch.empty(max_pairs, dtype=torch.int64, device=dev)
        f_len = torch.empty(max_pairs, dtype=torch.int32, device=dev)
        frame_pair = torch.empty(max_pairs, dtype=torch.int64, device=dev)
        n_frames = torch.empty((), dtype=torch.int64, device=dev)
        device.frames_compact(d_off, d_len, d_st, counts, f_off, f_len, frame_pair, n_frames, stream=stream)
        ifac = torch.empty((max_pairs, ifac_size), dtype=torch.uint8, device=dev)
        # with slots every frame (and the unmasked packet written at its
        # offset) has its token ciphertext on a line, and each plaintext,
        # written 16 B into its token's span, starts on one too
        pt_shift = 16 if aligned else 0
        if ifac_size:
            ifac_status = torch.empty(max_pairs, dtype=torch.int32, device=dev)
            p_len = torch.empty(max_pairs, dtype=torch.int32, device=dev)
            un = torch.empty_like(out)
            device.ifac_unmask(out, f_off, f_len, ifac_key, ifac, un, f_off, ifac_status, out_len=p_len,
                               stream=stream)
        else:
            # no IFAC on the interface: a packet with the IFAC flag set is
            # dropped, the others go to unpack as they are
            # (Transport.py:1482-1486); the empty entries past the frames
            # (f_len 0) stay dropped
            un = out
            # flag byte of each frame; entries past the frames (f_len 0, f_off
            # unspecified) are never read out of range and never count as flagged
            first = out[f_off.clamp(0, out.numel() - 1)]
            flagged = ((first & 0x80) != 0) & (f_len > 0)
            drop = flagged | (f_len <= 2)
            ifac_status = drop.to(torch.int32)
            p_len = torch.where(drop, torch.zeros_like(f_len), f_len)
        fields = torch.empty((max_pairs, 96), dtype=torch.uint8, device=dev)
        device.packet_unpack(un, f_off, p_len, fields, stream=stream)
        tok_off = torch.empty(max_pairs, dtype=torch.int64, device=dev)
        tok_len = torch.empty(max_pairs, dtype=torch.int32, device=dev)
        device.token_spans(fields, f_off, tok_off, tok_len, stream=stream)
        pt = torch.empty_like(un)
        pt_len = torch.empty(max_pairs, dtype=torch.int32, device=dev)
        status = torch.empty(max_pairs, dtype=torch.int32, device=dev)
        # each plaintext (at most its token's length - 48 bytes) is written inside its own token's span
        pt_off = tok_off + pt_shift if pt_shift else tok_off
        device.decrypt(ks, un, tok_off, tok_len, pt, pt_off, pt_len, status, stream=stream)
    return {"pt": pt, "pt_off": pt_off, "pt_len": pt_len, "status": status, "ifac": ifac,
            "ifac_status": ifac_status, "fields": fields, "frame_pair": frame_pair, "n_frames": n_frames,
            "frame_status": d_st, "frame_len": d_len, "counts": counts}


def _on(stream):
    """torch plumbing on the pipeline's stream (the device calls take it explicitly)."""
    return torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()
