// wire_kernels.hip — the wire-side neighbours of the token path.
//
// Inbound a node turns a byte stream from a socket into packets: HDLC
// deframing (TCPInterface.py:387-410), IFAC unmasking (Transport.py:1441-1475),
// header unpack and packet hash (Packet.py:236-268, 342-353), then the token
// decrypt.  Outbound is the mirror: header pack (Packet.py:167-228), token
// encrypt, IFAC masking (Transport.py:1069-1101), HDLC framing
// (TCPInterface.py:44-53, 323).  These are byte-granular, per-packet
// branchy transforms: one lane per packet (or per frame), HBM/latency-bound;
// the only SHA-heavy pieces are the IFAC mask (an HKDF stream as long as the
// packet) and the packet hash.
//
// Kernels:
//   k_scan_*         exclusive prefix sums (u64) for frame placement
//   k_hdlc_count     escaped frame length per packet
//   k_hdlc_write     7E || escape(packet) || 7E at its prefix-sum offset
//   k_flag_local / k_flag_gather    positions of every 7E in a stream
//   k_hdlc_unescape  one lane per consecutive flag pair: the read loop's two
//                    bytes.replace passes, check_frame_len, empty-frame skip
//   k_ifac           mask (outbound) / unmask (inbound) with HKDF(ifac, ifac_key)
//   k_unpack         header fields + SHA-256 packet hash
//   k_pack_headers   flags, hops, [transport id], destination hash, context
//   k_compact_*      the frames the read loop hands on, to the front in order
//   k_token_spans    each unpacked packet's data span (the token)
#include "token_device.h"
#include "token_launch.h"
#include "../../include/rnstok.h"

// IFAC mask/unmask: payload stores grouped by 64-B sector, as k_encrypt_split's
// ciphertext (round 6): node path, each build its own process, three runs each,
// outbound 2.632 -> 2.615 ms, inbound 3.260 -> 3.223 ms (profiles/r06_clock_ab/ifac_sector_ab.txt)
#ifndef RNSTOK_IFAC_ST_SECTOR
#define RNSTOK_IFAC_ST_SECTOR 1
#endif

namespace rnstok {

namespace {

constexpr uint8_t FLAG = 0x7E;      // HDLC flag; escapes are 7D x^0x20 (eqbytes constants below)
constexpr uint32_t HEADER_MINSIZE = 19, DST_LEN = 16, PATHFINDER_M = 128;
constexpr uint32_t SCAN_BLOCK = 1024;
constexpr uint32_t WAVE_GRID = 16384;        // workgroups of the wave-per-frame kernels (grid-stride beyond)

__device__ const uint32_t SHA_IV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                       0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

// ------------------------------------------------------------------ scan --

__device__ uint64_t block_exclusive_scan(uint64_t v, uint64_t *total) {
    __shared__ uint64_t sh[SCAN_BLOCK];
    const uint32_t t = threadIdx.x;
    sh[t] = v;
    __syncthreads();
    for (uint32_t d = 1; d < blockDim.x; d <<= 1) {
        const uint64_t add = t >= d ? sh[t - d] : 0;
        __syncthreads();
        sh[t] += add;
        __syncthreads();
    }
    const uint64_t incl = sh[t];
    *total = sh[blockDim.x - 1];
    __syncthreads();
    return incl - v;
}

__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_block(const uint64_t *in, uint64_t *out, uint64_t *part,
                                                           uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * SCAN_BLOCK + threadIdx.x;
    uint64_t tot;
    const uint64_t ex = block_exclusive_scan(i < n ? in[i] : 0, &tot);
    if (i < n) out[i] = ex;
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// one workgroup: exclusive scan of the block totals in place, total at part[nb]
__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_parts(uint64_t *part, uint64_t nb) {
    uint64_t carry = 0;
    for (uint64_t base = 0; base < nb; base += SCAN_BLOCK) {
        const uint64_t i = base + threadIdx.x;
        uint64_t tot;
        const uint64_t ex = block_exclusive_scan(i < nb ? part[i] : 0, &tot);
        if (i < nb) part[i] = ex + carry;
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) part[nb] = carry;
}

__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_add(uint64_t *out, const uint64_t *part, uint64_t n,
                                                         uint64_t *total_out) {
    const uint64_t i = (uint64_t)blockIdx.x * SCAN_BLOCK + threadIdx.x;
    if (i < n) out[i] += part[blockIdx.x];
    if (total_out && i == 0) *total_out = part[(n + SCAN_BLOCK - 1) / SCAN_BLOCK];
}

// ------------------------------------------------------- byte helpers --

// 0x80 in every byte of x equal to the byte replicated in c4 (exact: no borrow crosses bytes)
__device__ __forceinline__ uint32_t eqbytes(uint32_t x, uint32_t c4) {
    const uint32_t t = x ^ c4;
    return ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t | 0x7F7F7F7Fu);
}
__device__ __forceinline__ uint32_t escbytes(uint32_t x) { return eqbytes(x, 0x7E7E7E7Eu) | eqbytes(x, 0x7D7D7D7Du); }

// ------------------------------------------------------------- framing --
//
// One DPP row (16 lanes) per packet, 4 packets per wave: lane r of the row
// covers bytes [16r, 16r+16) of a 256-byte window with one 16-B load, so a
// wave keeps 4 packets' loads in flight (one wave per packet with 4-B lanes
// held one 500-B packet per wave and ran at 1.7-2.1 TB/s, latency-bound).
// Row sums and row prefix sums are DPP row_ror / row_shr adds.

template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, false);
}
// every lane of the 16-lane row gets the row's total
__device__ __forceinline__ uint32_t row_sum16(uint32_t x) {
    x += dpp<0x128>(x);     // row_ror:8
    x += dpp<0x124>(x);     // row_ror:4
    x += dpp<0x122>(x);     // row_ror:2
    x += dpp<0x121>(x);     // row_ror:1
    return x;
}
// inclusive prefix sum within the 16-lane row (row_shr reads 0 past the row start)
__device__ __forceinline__ uint32_t row_incl_scan16(uint32_t x) {
    x += dpp<0x111>(x);     // row_shr:1
    x += dpp<0x112>(x);     // row_shr:2
    x += dpp<0x114>(x);     // row_shr:4
    x += dpp<0x118>(x);     // row_shr:8
    return x;
}
// little-endian word of p[i, i+4), bytes at or past `end` read as 0
__device__ __forceinline__ uint32_t ld4_upto(const uint8_t *p, uint64_t i, uint64_t end) {
    if (i + 4 <= end) {
        uint32_t v;
        __builtin_memcpy(&v, p + i, 4);
        return v;
    }
    uint32_t v = 0;
    for (uint32_t k = 0; k < 4; ++k)
        if (i + k < end) v |= (uint32_t)p[i + k] << (8 * k);
    return v;
}
// 16 bytes of p[i, i+16), bytes at or past `end` read as 0.  (Loading the
// one or two aligned 16-B blocks that hold a partial window and shifting
// them into place was slower for framing and deframing alike, round 3:
// profiles/r03w_tail_ab/.)
__device__ __forceinline__ u32x4 ld16_upto(const uint8_t *p, uint64_t i, uint64_t end) {
    if (i + 16 <= end) return ld16(p + i);
    u32x4 v = {ld4_upto(p, i, end), ld4_upto(p, i + 4, end), ld4_upto(p, i + 8, end), ld4_upto(p, i + 12, end)};
    return v;
}
__device__ __forceinline__ uint32_t esc_count16(u32x4 v) {
    return __builtin_popcount(escbytes(v.x)) + __builtin_popcount(escbytes(v.y)) + __builtin_popcount(escbytes(v.z)) +
           __builtin_popcount(escbytes(v.w));
}

// v_perm selector tables for the escape-dense lanes (S0 = data word,
// S1 = 0x7D7D7D7D; selector bytes 0-3 pick S1, 4-7 pick S0, 0x0C gives 0):
//   expand[p]:  the word's bytes with "7D" inserted before each byte whose
//               bit is set in the 4-bit pattern p (lo, hi: 8 output bytes)
//   compact[p]: the bytes whose bit is set in p, in order
struct SelTables {
    uint32_t expand[16][2];
    uint32_t compact[16];
};
__device__ __forceinline__ void fill_sel_tables(SelTables *t) {
    if (threadIdx.x < 16u) {
        const uint32_t p = threadIdx.x;
        uint32_t seq[8], m = 0, c[4], mc = 0;
        for (uint32_t k = 0; k < 4; ++k) {
            if ((p >> k) & 1u) {
                seq[m++] = 0u;
                c[mc++] = 4u + k;
            }
            seq[m++] = 4u + k;
        }
        while (m < 8) seq[m++] = 0x0Cu;
        while (mc < 4) c[mc++] = 0x0Cu;
        t->expand[p][0] = seq[0] | seq[1] << 8 | seq[2] << 16 | seq[3] << 24;
        t->expand[p][1] = seq[4] | seq[5] << 8 | seq[6] << 16 | seq[7] << 24;
        t->compact[p] = c[0] | c[1] << 8 | c[2] << 16 | c[3] << 24;
    }
    __syncthreads();
}
// 4-bit pattern of the bytes flagged 0x80 in m (bit k = byte k)
__device__ __forceinline__ uint32_t byte_pattern(uint32_t m) {
    return ((((m >> 7) & 0x01010101u) * 0x01020408u) >> 24) & 0xFu;
}

// exactly k (0..16) bytes of lo||hi at d: a 16-B store, or 8/4/2/1-byte pieces
__device__ __forceinline__ void st_exact16(uint8_t *d, uint64_t lo, uint64_t hi, uint32_t k) {
    if (k == 16u) {
        st16(d, u32x4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)});
        return;
    }
    if (k >= 8u) {
        __builtin_memcpy(d, &lo, 8);
        d += 8; k -= 8u; lo = hi;
    }
    if (k >= 4u) {
        const uint32_t w = (uint32_t)lo;
        __builtin_memcpy(d, &w, 4);
        d += 4; k -= 4u; lo >>= 32;
    }
    if (k >= 2u) {
        const uint16_t w = (uint16_t)lo;
        __builtin_memcpy(d, &w, 2);
        d += 2; k -= 2u; lo >>= 16;
    }
    if (k) *d = (uint8_t)lo;
}
// own (the first t < 16 bytes of lo||hi, the rest 0) followed by the first
// 16 - t bytes of nlo||nhi
__device__ __forceinline__ void funnel16(uint64_t &lo, uint64_t &hi, uint64_t nlo, uint64_t nhi, uint32_t t) {
    if (t < 8u) {
        const uint32_t r = 8u * t;
        hi = t ? (nlo >> (64u - r)) | (nhi << r) : nhi;
        lo |= t ? nlo << r : nlo;
    } else if (t == 8u) {
        hi = nlo;
    } else {
        hi |= nlo << (8u * (t - 8u));
    }
}

__global__ __launch_bounds__(256) void k_hdlc_count(const uint8_t *pkt, const uint64_t *off, const uint32_t *len,
                                                    uint64_t *flen, uint32_t n) {
    const uint32_t lane = threadIdx.x & 63u, rl = lane & 15u;
    const uint32_t g0 = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, ng = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t g = g0; 4ull * g < n; g += ng) {
        const uint32_t i = 4u * g + (lane >> 4);
        const bool valid = i < n;
        const uint8_t *p = pkt + (valid ? off[i] : 0);
        const uint32_t L = valid ? len[i] : 0u;
        uint32_t extra = 0;
        for (uint32_t b = 16u * rl; b < L; b += 256u) extra += esc_count16(ld16_upto(p, b, L));
        extra = row_sum16(extra);
        if (rl == 0 && valid) flen[i] = 2ull + L + extra;     // 7E || escape(p) || 7E
    }
}

__global__ __launch_bounds__(256) void k_hdlc_write(const uint8_t *pkt, const uint64_t *off, const uint32_t *len,
                                                    const uint64_t *foff, uint8_t *out, uint32_t n) {
    __shared__ SelTables tab;
    fill_sel_tables(&tab);
    const uint32_t lane = threadIdx.x & 63u, rl = lane & 15u;
    const uint32_t g0 = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, ng = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t g = g0; 4ull * g < n; g += ng) {
        const uint32_t i = 4u * g + (lane >> 4);
        const bool valid = i < n;
        const uint8_t *p = pkt + (valid ? off[i] : 0);
        uint8_t *o = out + (valid ? foff[i] : 0);
        const uint32_t L = valid ? len[i] : 0u;
        if (rl == 0 && valid) o[0] = FLAG;
        uint64_t base = 1;                       // output position of the window's first byte
        // rows run as many windows as their own packet needs; the DPP ops
        // below read only lanes of the same row, which share the trip count
        // the next window's load is in flight while this one is placed
        u32x4 vn = 16u * rl < L ? ld16_upto(p, 16u * rl, L) : u32x4{0u, 0u, 0u, 0u};
        for (uint32_t w = 0; w < L; w += 256u) {
            const uint32_t b = w + 16u * rl;
            const uint32_t nb = b < L ? min(16u, L - b) : 0u;
            const u32x4 v = vn;
            vn = b + 256u < L ? ld16_upto(p, b + 256u, L) : u32x4{0u, 0u, 0u, 0u};
            const uint32_t esc = esc_count16(v);
            const uint32_t sz = nb + esc;
            const uint32_t incl = row_incl_scan16(sz);
            uint8_t *q = o + base + (incl - sz);
            // HDLC.escape (TCPInterface.py:50-52: ESC first, then FLAG; per
            // byte the same: 7D x^0x20): each word expands through one
            // selector pair into 4..8 bytes; the lane's sz expanded bytes are
            // packed in a[0..3] with 64-bit shifts.  Stores are row-wide as in
            // unescape: 16 B at q, and the rest (sz - 16 bytes) completed with
            // the next lane's first output bytes, which that lane stores too
            // with the same values; the row's last lane and a packet's last
            // lane store exactly.  (The per-word form, every word of an escaping
            // lane stored as a dword plus single bytes, was 6 % slower:
            // profiles/r03x_frame_ab/.)
            uint64_t a[4] = {((uint64_t)v.y << 32) | v.x, ((uint64_t)v.w << 32) | v.z, 0ull, 0ull};
            if (esc) {
                const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
                a[0] = a[1] = 0ull;
                uint32_t at = 0;
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j) {
                    const uint32_t e = escbytes(wv[j]);                // bytes past nb are 0: never escape
                    const uint32_t pat = byte_pattern(e);
                    const uint32_t x = wv[j] ^ (e >> 2);               // 0x80 -> 0x20 in the escaped bytes
                    const uint64_t piece = ((uint64_t)__builtin_amdgcn_perm(x, 0x7D7D7D7Du, tab.expand[pat][1]) << 32) |
                                           __builtin_amdgcn_perm(x, 0x7D7D7D7Du, tab.expand[pat][0]);
                    const uint32_t k = at >> 3, r = 8u * (at & 7u);
                    const uint64_t pl = piece << r, ph = r ? piece >> (64u - r) : 0ull;
#pragma unroll
                    for (uint32_t i = 0; i < 4; ++i) a[i] |= (i == k ? pl : 0ull) | (i == k + 1u ? ph : 0ull);
                    at += 4u * j < nb ? min(4u, nb - 4u * j) + __builtin_popcount(e) : 0u;
                }
            }
            // the next lane's first 16 output bytes and its size (row_shl:1; the row's last lane reads 0)
            const uint64_t n0 = ((uint64_t)dpp<0x101>((uint32_t)(a[0] >> 32)) << 32) | dpp<0x101>((uint32_t)a[0]);
            const uint64_t n1 = ((uint64_t)dpp<0x101>((uint32_t)(a[1] >> 32)) << 32) | dpp<0x101>((uint32_t)a[1]);
            const uint32_t szn = dpp<0x101>(sz);
            if (sz >= 16u) {
                st16(q, u32x4{(uint32_t)a[0], (uint32_t)(a[0] >> 32), (uint32_t)a[1], (uint32_t)(a[1] >> 32)});
                const uint32_t t = sz - 16u;
                if (t == 16u || (t && rl != 15u && szn >= 16u - t)) {
                    uint64_t lo = a[2], hi = a[3];
                    if (t < 16u) funnel16(lo, hi, n0, n1, t);
                    st16(q + 16, u32x4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)});
                } else if (t) {
                    st_exact16(q + 16, a[2], a[3], t);
                }
            } else if (sz) {
                st_exact16(q, a[0], a[1], sz);
            }
            base += row_sum16(sz);
        }
        if (rl == 0 && valid) o[base] = FLAG;
    }
}

// ----------------------------------------------------------- deframing --

constexpr uint32_t FLAG_CHUNK = 16384;       // stream bytes per workgroup (256 threads x 64)

// wave-wide inclusive prefix sum: row scans, then the lower rows' totals
// (readlane) added in
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x = row_incl_scan16(x);
    const uint32_t r0 = __builtin_amdgcn_readlane(x, 15), r1 = __builtin_amdgcn_readlane(x, 31),
                   r2 = __builtin_amdgcn_readlane(x, 47);
    const uint32_t lane = threadIdx.x & 63u;
    return x + (lane >= 16u ? r0 : 0u) + (lane >= 32u ? r1 : 0u) + (lane >= 48u ? r2 : 0u);
}

// Flag positions within each chunk, in stream order, and the chunk's flag
// count: the one pass over the stream (k_flag_gather places them once the
// counts are scanned; a separate counting pass read the stream a second
// time).  Thread t loads the 16-B units t, t+256, t+512, t+768 of its chunk
// (each load instruction 1 KiB contiguous across a wave); the stream-order rank of a unit's flags is the
// block's flags in the earlier 4 KiB quarters plus those of the lower threads
// in its own quarter: the four per-thread counts (<= 16 each, <= 4096 per
// block) ride as 16-bit fields of two words through one wave scan each and
// one LDS exchange of the wave totals.  The form with 64 contiguous bytes
// per thread loaded at a 64-B lane stride and ranked with an 8-step LDS scan
// (16 barriers): 137 against 111 us, profiles/r03t_deframe_ab/.
__global__ __launch_bounds__(256) void k_flag_local(const uint8_t *buf, uint64_t len, uint64_t *cnt, uint16_t *loc) {
    const uint64_t cbase = (uint64_t)blockIdx.x * FLAG_CHUNK;
    const uint32_t t = threadIdx.x, wave = t >> 6;
    uint32_t m[4][4], c[4];
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        const uint64_t u = cbase + 4096ull * k + 16ull * t;
        const u32x4 v = u < len ? ld16_upto(buf, u, len) : u32x4{0u, 0u, 0u, 0u};
        m[k][0] = eqbytes(v.x, 0x7E7E7E7Eu); m[k][1] = eqbytes(v.y, 0x7E7E7E7Eu);
        m[k][2] = eqbytes(v.z, 0x7E7E7E7Eu); m[k][3] = eqbytes(v.w, 0x7E7E7E7Eu);
        c[k] = __builtin_popcount(m[k][0]) + __builtin_popcount(m[k][1]) + __builtin_popcount(m[k][2]) +
               __builtin_popcount(m[k][3]);
    }
    const uint32_t lo = c[0] | c[1] << 16, hi = c[2] | c[3] << 16;
    const uint32_t ilo = wave_incl_scan(lo), ihi = wave_incl_scan(hi);
    __shared__ uint32_t wtot[2][4];
    if ((t & 63u) == 63u) {
        wtot[0][wave] = ilo;
        wtot[1][wave] = ihi;
    }
    __syncthreads();
    uint32_t plo = 0, phi = 0, tlo = 0, thi = 0;
#pragma unroll
    for (uint32_t w = 0; w < 4; ++w) {
        const uint32_t a = wtot[0][w], b = wtot[1][w];
        plo += w < wave ? a : 0u;
        phi += w < wave ? b : 0u;
        tlo += a;
        thi += b;
    }
    const uint32_t elo = plo + ilo - lo, ehi = phi + ihi - hi;
    const uint32_t excl[4] = {elo & 0xFFFFu, elo >> 16, ehi & 0xFFFFu, ehi >> 16};
    const uint32_t tot[4] = {tlo & 0xFFFFu, tlo >> 16, thi & 0xFFFFu, thi >> 16};
    uint16_t *out = loc + (uint64_t)blockIdx.x * FLAG_CHUNK;
    if (t == 0) cnt[blockIdx.x] = tot[0] + tot[1] + tot[2] + tot[3];
    uint32_t before = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        if (c[k]) {
            uint32_t w = before + excl[k];
            const uint32_t u = 4096u * k + 16u * t;
            for (uint32_t j = 0; j < 4; ++j)
                for (uint32_t f = m[k][j]; f; f &= f - 1) out[w++] = (uint16_t)(u + 4 * j + (__builtin_ctz(f) >> 3));
        }
        before += tot[k];
    }
}

// Stream-order flag positions: chunk c's count[c] local positions (from
// k_flag_local) go to pos[cnt_off[c] + part[c / SCAN_BLOCK] ...], one wave per
// chunk.
__global__ __launch_bounds__(256) void k_flag_gather(const uint64_t *cnt, const uint64_t *cnt_off, const uint64_t *part,
                                                     const uint16_t *loc, uint64_t chunks, uint64_t *pos) {
    const uint64_t c = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (c >= chunks) return;
    const uint32_t lane = threadIdx.x & 63u, n = (uint32_t)cnt[c];
    const uint64_t base = cnt_off[c] + part[c / SCAN_BLOCK], cb = c * FLAG_CHUNK;
    const uint16_t *l = loc + cb;
    for (uint32_t i = lane; i < n; i += 64u) pos[base + i] = cb + l[i];
}

// One DPP row (16 lanes x 16 B) per consecutive flag pair (k, k+1), 4 pairs
// per wave: the read loop's frame buf[pos_k+1 : pos_{k+1}) with its two
// bytes.replace passes (TCPInterface.py:397-398: ESC,5E -> 7E first, then
// ESC,5D -> 7D, each left to right and non-overlapping), written at
// out + pos_k + 1.  Neither pattern can overlap itself and a 7D is never the
// byte a replacement removes, so the two passes are one local rule on the
// input bytes: byte i is dropped when byte i-1 is 7D and byte i is 5E or 5D;
// a 7D followed by 5E becomes 7E.  Evaluated on whole words (eqbytes on the
// words shifted by one byte); the byte before a frame is its opening flag and
// the byte after it the closing flag, so neither rule fires across the frame
// edge.  Kept bytes are placed with a row prefix sum.
__device__ void deframe_counts(const uint64_t *nflags_p, const uint64_t *pos, uint64_t len, uint32_t hw_mtu,
                               uint64_t *counts);
__global__ __launch_bounds__(256) void k_hdlc_unescape(const uint8_t *buf, uint64_t len, const uint64_t *pos,
                                                       const uint64_t *nflags_p, uint64_t max_pairs, uint32_t hw_mtu,
                                                       uint32_t ifac_size, uint8_t *out, uint64_t *frame_off,
                                                       uint32_t *frame_len, int32_t *status, uint64_t *counts,
                                                       uint32_t line_phase) {
    __shared__ SelTables tab;
    // the pair count and the bytes consumed (k_deframe_counts' job, folded in: one launch fewer)
    if (blockIdx.x == 0 && threadIdx.x == 0) deframe_counts(nflags_p, pos, len, hw_mtu, counts);
    fill_sel_tables(&tab);
    const uint64_t nf = *nflags_p;
    uint64_t npairs = nf > 1 ? nf - 1 : 0;
    if (npairs > max_pairs) npairs = max_pairs;
    const uint32_t lane = threadIdx.x & 63u, rl = lane & 15u;
    const uint64_t g0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, ng = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    // Each row takes two consecutive flag pairs: a Reticulum stream alternates
    // frames with the empty 7E|7E gaps between them, and with one pair per
    // row every other row idled on a gap (unescape 546 -> 459 us, A/B in
    // profiles/r02av_unesc_pair2_ab.txt).
    constexpr uint32_t PPR = 2;
    for (uint64_t g = g0; 4 * PPR * g < npairs; g += ng) {
      for (uint32_t sub = 0; sub < PPR; ++sub) {
        const uint64_t k = 4 * PPR * g + PPR * (lane >> 4) + sub;
        const bool valid = k < npairs;
        const uint64_t a = valid ? pos[k] + 1 : 0, e = valid ? pos[k + 1] : 0;
        // slots (line_phase < 128): frame k at the first offset >= a + 128 k
        // whose byte line_phase starts a 128-B line; frames never overlap,
        // since each moves by less than 128 B more than the one before it
        uint64_t ao = a;
        if (line_phase < 128u) {
            ao = a + 128ull * k;
            ao += (0ull - ((uint64_t)(uintptr_t)out + ao + line_phase)) & 127ull;
        }
        uint8_t *o = out + ao;
        uint64_t kept_total = 0;
        uint32_t carry = FLAG;                    // the byte before the window: the opening flag first
        for (uint64_t w = a; w < e; w += 256u) {
            const uint64_t b = w + 16u * rl;
            const uint32_t nb = b < e ? (uint32_t)min((uint64_t)16, e - b) : 0u;
            // a window's last lane: one 16-B load with the bytes past the
            // frame masked off, unless the load would run past the stream
            // (the byte-wise form issues up to 15 loads one after another)
            u32x4 v = u32x4{0u, 0u, 0u, 0u};
            if (nb == 16u || (nb && b + 16u <= len)) {
                v = ld16(buf + b);
                if (nb < 16u) {
                    uint64_t lo = ((uint64_t)v.y << 32) | v.x, hi = ((uint64_t)v.w << 32) | v.z;
                    if (nb <= 8u) {
                        hi = 0;
                        lo = nb == 8u ? lo : lo & ((1ull << (8u * nb)) - 1ull);
                    } else {
                        hi &= (1ull << (8u * (nb - 8u))) - 1ull;
                    }
                    v = u32x4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
                }
            } else if (nb) {
                v = ld16_upto(buf, b, e);
            }
            uint32_t prevb = dpp<0x111>(v.w) >> 24;          // row_shr:1: the previous lane's last byte
            if (rl == 0) prevb = carry;
            uint32_t nextb = dpp<0x101>(v.x) & 0xFFu;         // row_shl:1: the next lane's first byte
            // (prefetching the next window instead of this byte load: +3.5 %, measured)
            if (rl == 15) nextb = b + 16 < e ? buf[b + 16] : 0u;
            const uint32_t x[4] = {v.x, v.y, v.z, v.w};
            uint32_t y[4], drop[4], ndrop = 0;
            // Each byte test once per word (7D, 5E, 5D: 0x80 per matching
            // byte), the neighbour's test by shifting the FLAG words by one
            // byte across the word and lane edges (the byte before the lane's
            // first is prevb, the byte after its last nextb) instead of
            // testing shifted data words again: 3 tests per word, not 5.
            uint32_t e7d[4], e5e[4], e5d[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                e7d[j] = eqbytes(x[j], 0x7D7D7D7Du);
                e5e[j] = eqbytes(x[j], 0x5E5E5E5Eu);
                e5d[j] = eqbytes(x[j], 0x5D5D5D5Du);
            }
            const uint32_t prev7d = prevb == 0x7Du ? 0x80000000u : 0u, next5e = nextb == 0x5Eu ? 0x80u : 0u;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t p7 = __builtin_amdgcn_alignbit(e7d[j], j ? e7d[j - 1] : prev7d, 24);   // byte i-1 is 7D
                const uint32_t n5 = __builtin_amdgcn_alignbit(j < 3 ? e5e[j + 1] : next5e, e5e[j], 8); // byte i+1 is 5E
                drop[j] = p7 & (e5e[j] | e5d[j]);
                const uint32_t conv = e7d[j] & n5;
                y[j] = x[j] ^ ((conv >> 7) * 3u);                                                     // 7D -> 7E
                ndrop += __builtin_popcount(drop[j]);
            }
            const uint32_t kept = nb - ndrop;
            const uint32_t incl = row_incl_scan16(kept);
            uint8_t *q = o + kept_total + (incl - kept);
            // Row-wide 16-B stores.  The lane's kept bytes are packed low in
            // c[0..3] (each word through its compaction selector, the pieces
            // placed with 64-bit shifts).  A lane then stores 16 bytes at its
            // output position: its own kept bytes followed by the next lane's
            // first 16 - kept, which that lane stores too, with the same
            // values, so the overlap is benign; nothing past the row's output
            // is written.  Lanes that cannot borrow enough from their
            // neighbour (the row's last lane, the frame's last lane, lanes
            // with fewer than 8 kept bytes) store exactly their bytes.  The
            // per-word form stored every word of an escape-holding lane as a dword
            // plus single bytes: 459 against 368 us, profiles/r03s_unesc_ab/.
            uint32_t c[4] = {y[0], y[1], y[2], y[3]};
            if (kept != 16u) {
                uint64_t lo = 0, hi = 0;
                uint32_t at = 0;
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j) {
                    const uint32_t m = nb > 4u * j ? min(4u, nb - 4u * j) : 0u;
                    const uint32_t keep = byte_pattern(~drop[j] & 0x80808080u) & ((1u << m) - 1u);
                    const uint64_t piece = __builtin_amdgcn_perm(y[j], 0u, tab.compact[keep]);
                    if (at < 8u) {
                        lo |= piece << (8u * at);
                        if (at > 4u) hi |= piece >> (8u * (8u - at));
                    } else {
                        hi |= piece << (8u * (at - 8u));
                    }
                    at += __builtin_popcount(keep);
                }
                c[0] = (uint32_t)lo; c[1] = (uint32_t)(lo >> 32); c[2] = (uint32_t)hi; c[3] = (uint32_t)(hi >> 32);
            }
            // the next lane's first 8 kept bytes and its count (row_shl:1; the row's last lane reads 0)
            const uint32_t n0 = dpp<0x101>(c[0]), n1 = dpp<0x101>(c[1]), kn = dpp<0x101>(kept);
            const uint64_t up = ((uint64_t)c[3] << 32) | c[2];
            if (rl != 15u && kept >= 8u && kept + kn >= 16u) {
                const uint32_t t = kept - 8u;       // own bytes in the upper half: 0..8
                const uint64_t nx = ((uint64_t)n1 << 32) | n0;
                const uint64_t w = t == 8u ? up : ((up & ((1ull << (8u * t)) - 1ull)) | (nx << (8u * t)));
                st16(q, u32x4{c[0], c[1], (uint32_t)w, (uint32_t)(w >> 32)});
            } else if (kept == 16u) {
                st16(q, u32x4{c[0], c[1], c[2], c[3]});
            } else if (kept) {
                uint64_t v64 = ((uint64_t)c[1] << 32) | c[0];
                uint32_t k = kept;
                uint8_t *d = q;
                if (k >= 8u) {
                    __builtin_memcpy(d, &v64, 8);
                    d += 8; k -= 8u; v64 = up;
                }
                if (k >= 4u) {
                    const uint32_t w4 = (uint32_t)v64;
                    __builtin_memcpy(d, &w4, 4);
                    d += 4; k -= 4u; v64 >>= 32;
                }
                if (k >= 2u) {
                    const uint16_t w2 = (uint16_t)v64;
                    __builtin_memcpy(d, &w2, 2);
                    d += 2; k -= 2u; v64 >>= 16;
                }
                if (k) *d = (uint8_t)v64;
            }
            kept_total += row_sum16(kept);
            carry = row_sum16(rl == 15 ? v.w >> 24 : 0u);      // the window's last byte, to every lane
        }
        if (rl == 0 && valid) {
            frame_off[k] = ao;
            frame_len[k] = (uint32_t)kept_total;
            // check_frame_len (TCPInterface.py:336-339); empty frames are skipped (:400)
            status[k] = kept_total == 0 ? RT_FRAME_EMPTY
                                        : ((kept_total <= HEADER_MINSIZE || kept_total > (uint64_t)hw_mtu + ifac_size)
                                               ? RT_FRAME_BAD_LEN
                                               : RT_FRAME_OK);
        }
      }
    }
}

__device__ __forceinline__ void deframe_counts(const uint64_t *nflags_p, const uint64_t *pos, uint64_t len,
                                               uint32_t hw_mtu, uint64_t *counts) {
    const uint64_t nf = *nflags_p;
    counts[0] = nf > 1 ? nf - 1 : 0;
    // What the loop keeps for the next read (TCPInterface.py:391-411): after a
    // pair it has cut the buffer at the pair's closing flag, so it holds the
    // buffer from the last flag on; with a single flag it never cut it and
    // holds everything, junk before the flag included.  It drops what it
    // holds once that is longer than 2*HW_MTU (:406-407), and all of it when
    // there is no flag (:408-410).
    uint64_t consumed = len;
    if (nf == 1) {
        consumed = len > 2ull * hw_mtu ? len : 0;
    } else if (nf > 1) {
        const uint64_t last = pos[nf - 1];
        consumed = (len - last > 2ull * hw_mtu) ? len : last;
    }
    counts[1] = consumed;
}
__global__ void k_deframe_counts(const uint64_t *nflags_p, const uint64_t *pos, uint64_t len, uint32_t hw_mtu,
                                 uint64_t *counts) {
    deframe_counts(nflags_p, pos, len, hw_mtu, counts);
}

// ------------------------------------------------------------------ IFAC --

// HMAC midstates for a <= 64-byte key given as bytes
__device__ __forceinline__ void key_midstates(const uint8_t *key, uint32_t klen, uint32_t hi[8], uint32_t ho[8]) {
    uint32_t wi[16], wo[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        uint32_t v = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t q = 4u * k + j;
            v = (v << 8) | (q < klen ? key[q] : 0u);
        }
        wi[k] = v ^ 0x36363636u;
        wo[k] = v ^ 0x5c5c5c5cu;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) hi[k] = ho[k] = SHA_IV[k];
    sha256_compress(hi, wi);
    sha256_compress(ho, wo);
}

// One lane per packet.  Outbound (MASK): new_raw = [raw0|0x80, raw1] || ifac ||
// raw[2:], masked with HKDF(len+ifac_size, ifac, ifac_key) except the IFAC
// bytes, byte 0 keeps the flag (Transport.py:1069-1101).  Inbound: the IFAC
// is raw[2:2+n], mask = HKDF(len, ifac, ifac_key) over everything but the
// IFAC, reassembled [un0 & 0x7f, un1] || un[2+n:] (Transport.py:1441-1475).
template <bool MASK>
__global__ __attribute__((amdgpu_waves_per_eu(4, 4))) __launch_bounds__(256) void k_ifac(IfacArgs a) {
    // the ifac_key midstates are the same for every packet: wave 0 computes
    // them once per workgroup (2 of a 500-B packet's 38 compressions)
    __shared__ uint32_t key_ms[16];
    if (threadIdx.x < 64u) {
        uint32_t ki[8], ko[8];
        key_midstates(a.ifac_key, a.key_len, ki, ko);
        if (threadIdx.x == 0u) {
#pragma unroll
            for (int k = 0; k < 8; ++k) { key_ms[k] = ki[k]; key_ms[8 + k] = ko[k]; }
        }
    }
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const uint8_t *raw = a.pkt + a.pkt_off[i];
    const uint32_t L = a.pkt_len[i], n = a.ifac_size;
    uint8_t *o = a.out + a.out_off[i];
    const uint8_t *ifac;
    if (MASK) {
        ifac = a.ifac + (uint64_t)i * n;
    } else {
        // len(raw) > 2, IFAC flag set, len(raw) > 2 + ifac_size (:1441-1445)
        const bool ok = L > 2u && (raw[0] & 0x80u) && L > 2u + n;
        a.status[i] = ok ? 0 : 1;
        if (a.out_len) a.out_len[i] = ok ? L - n : 0u;
        if (!ok) return;
        ifac = raw + 2;
        for (uint32_t k = 0; k < n; ++k) a.ifac[(uint64_t)i * n + k] = ifac[k];
    }
    const uint32_t total = MASK ? L + n : L;           // HKDF output length
    // HKDF (HKDF.py:35-62) with salt = ifac_key, ikm = ifac, no context:
    // PRK = HMAC(ifac_key, ifac); T_b = HMAC(PRK, T_{b-1} || b+1)
    uint32_t phi[8], pho[8];
    if constexpr (MASK) {
        // PRK's blocks, its outer hash and PRK's two key midstates through ONE
        // inlined compression (steps uniform across the wave: scalar branches):
        // 4 % faster for the mask, 1.7 % slower for the unmask, whose early
        // exit makes the steps divergent (profiles/r03as_ifac_site_ab/)
        const uint64_t bits = (64ull + n) * 8ull;
        const uint32_t nblk = (n + 8u) / 64u + 1u;
        uint32_t st[8], prk[8];
#pragma nounroll
        for (uint32_t s = 0; s < nblk + 3u; ++s) {
            uint32_t w[16], h[8];
            if (s < nblk) {                       // PRK inner: ipad midstate, then the IFAC's blocks
#pragma unroll
                for (int k = 0; k < 8; ++k) h[k] = s == 0 ? key_ms[k] : st[k];
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    uint32_t v = 0;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const uint32_t q = 64u * s + 4u * k + j;
                        v = (v << 8) | (q < n ? ifac[q] : (q == n ? 0x80u : 0u));
                    }
                    w[k] = v;
                }
                if (s + 1 == nblk) {
                    w[14] = (uint32_t)(bits >> 32);
                    w[15] = (uint32_t)bits;
                }
            } else if (s == nblk) {               // PRK outer: opad midstate, inner digest
#pragma unroll
                for (int k = 0; k < 8; ++k) { h[k] = key_ms[8 + k]; w[k] = st[k]; }
                w[8] = 0x80000000u;
#pragma unroll
                for (int k = 9; k < 15; ++k) w[k] = 0;
                w[15] = (64 + 32) * 8;
            } else {                              // PRK ^ ipad, PRK ^ opad
                const uint32_t pad = s == nblk + 1u ? 0x36363636u : 0x5c5c5c5cu;
#pragma unroll
                for (int k = 0; k < 8; ++k) { h[k] = SHA_IV[k]; w[k] = prk[k] ^ pad; w[8 + k] = pad; }
            }
            sha256_compress(h, w);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if (s < nblk) st[k] = h[k];
                else if (s == nblk) prk[k] = h[k];
                else if (s == nblk + 1u) phi[k] = h[k];
                else pho[k] = h[k];
            }
        }
    } else {
        uint32_t hi[8], ho[8], prk[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) { hi[k] = key_ms[k]; ho[k] = key_ms[8 + k]; }
        {
            uint32_t w[16], h[8];
            // ifac_size <= 64: one or two message blocks after the ipad block
            const uint64_t bits = (64ull + n) * 8ull;
            const uint32_t nblk = (n + 8u) / 64u + 1u;
#pragma unroll
            for (int k = 0; k < 8; ++k) h[k] = hi[k];
            for (uint32_t b = 0; b < nblk; ++b) {
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    uint32_t v = 0;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const uint32_t q = 64u * b + 4u * k + j;
                        v = (v << 8) | (q < n ? ifac[q] : (q == n ? 0x80u : 0u));
                    }
                    w[k] = v;
                }
                if (b + 1 == nblk) {
                    w[14] = (uint32_t)(bits >> 32);
                    w[15] = (uint32_t)bits;
                }
                sha256_compress(h, w);
            }
            hmac_outer(prk, h, ho);
        }
        uint8_t prkb[32];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            prkb[4 * k] = prk[k] >> 24; prkb[4 * k + 1] = prk[k] >> 16; prkb[4 * k + 2] = prk[k] >> 8; prkb[4 * k + 3] = prk[k];
        }
        key_midstates(prkb, 32, phi, pho);
    }
    uint32_t t[8];
    // RNSTOK_IFAC_ST_SECTOR: payload units are stored by 64-B sector in one
    // burst (as k_encrypt_split's ciphertext): units of a sector the next
    // chunk completes are held (up to 3: h0..h2 at hdst + 16 k)
    u32x4 h0 = {0u, 0u, 0u, 0u}, h1 = h0, h2 = h0;
    uint8_t *hdst = nullptr;
    uint32_t nh = 0;
    for (uint32_t b = 0; 32u * b < total; ++b) {
        // message T_{b-1} (32 B, none for b = 0) || counter byte
        uint32_t w[16], h[8];
#pragma unroll
        for (int k = 0; k < 16; ++k) w[k] = 0;
        if (b == 0) {
            w[0] = ((b + 1u) & 255u) << 24 | 0x800000u;
            w[15] = (64u + 1u) * 8u;
        } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) w[k] = t[k];
            w[8] = ((b + 1u) & 255u) << 24 | 0x800000u;
            w[15] = (64u + 33u) * 8u;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) h[k] = phi[k];
        sha256_compress(h, w);
        hmac_outer(t, h, pho);
        // mask bytes 32b .. 32b+31 of the (masked) packet
        const uint32_t lo = 32u * b;
        if (lo >= 2u + n && lo + 32u <= total) {
            // inside the payload: 2 x 16 B, masked in place of the byte loop below
            const u32x4 m0 = {bswap(t[0]), bswap(t[1]), bswap(t[2]), bswap(t[3])};
            const u32x4 m1 = {bswap(t[4]), bswap(t[5]), bswap(t[6]), bswap(t[7])};
            const uint8_t *src = MASK ? raw + (lo - n) : raw + lo;
            uint8_t *dst = MASK ? o + lo : o + (lo - n);
            const u32x4 d0 = ld16(src) ^ m0, d1 = ld16(src + 16) ^ m1;
            if (RNSTOK_IFAC_ST_SECTOR) {
                // phases of d0 / d1 in their 64-B sector; held units precede d0
                const uint32_t ph = ((uint32_t)(uintptr_t)dst >> 4) & 3u;
                if (ph == 2u || ph == 3u) {            // d0 (and d1 at phase 3) closes the open sector
                    if (nh > 0u) st16(hdst, h0);
                    if (nh > 1u) st16(hdst + 16, h1);
                    if (nh > 2u) st16(hdst + 32, h2);
                    st16(dst, d0);
                    if (ph == 2u) {
                        st16(dst + 16, d1);
                        nh = 0u;
                    } else {
                        h0 = d1; hdst = dst + 16; nh = 1u;
                    }
                } else {                              // phases 0/1: the sector closes with the next chunk
                    if (nh == 0u) { h0 = d0; h1 = d1; hdst = dst; nh = 2u; }
                    else { h1 = d0; h2 = d1; nh = 3u; }
                }
            } else {
                st16(dst, d0);
                st16(dst + 16, d1);
            }
            continue;
        }
        if (RNSTOK_IFAC_ST_SECTOR && nh) {            // the tail's bytes follow: flush the held units
            st16(hdst, h0);
            if (nh > 1u) st16(hdst + 16, h1);
            if (nh > 2u) st16(hdst + 32, h2);
            nh = 0u;
        }
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            const uint32_t pos = lo + j;
            if (pos >= total) continue;
            const uint8_t m = (uint8_t)(t[j >> 2] >> (24 - 8 * (j & 3)));
            if (MASK) {
                uint8_t v;
                if (pos == 0) v = (uint8_t)(((raw[0] | 0x80u) ^ m) | 0x80u);
                else if (pos == 1) v = raw[1] ^ m;
                else if (pos < 2u + n) v = ifac[pos - 2];                 // the IFAC itself is not masked
                else v = raw[pos - n] ^ m;
                o[pos] = v;
            } else {
                // reassembled: [un0 & 0x7f, un1] || un[2+n:]
                if (pos == 0) o[0] = (uint8_t)((raw[0] ^ m) & 0x7Fu);
                else if (pos == 1) o[1] = raw[1] ^ m;
                else if (pos >= 2u + n) o[pos - n] = raw[pos] ^ m;
            }
        }
    }
    if (RNSTOK_IFAC_ST_SECTOR && nh) {
        st16(hdst, h0);
        if (nh > 1u) st16(hdst + 16, h1);
        if (nh > 2u) st16(hdst + 32, h2);
    }
}

// ------------------------------------------------------ frame compaction --
//
// The frames a read hands to Transport (TCPInterface.py:391-401: pair k <
// counts[0] with status RT_FRAME_OK), in stream order, at the front of the
// per-frame arrays; one pair per thread, SCAN_BLOCK per workgroup.  Pass 1
// counts each block's frames, k_scan_parts places the blocks, pass 2 writes
// the frames and clears the entries past the last one.
__device__ __forceinline__ bool handed_on(const int32_t *st, uint64_t pairs, uint64_t k) {
    return k < pairs && st[k] == RT_FRAME_OK;
}

__global__ __launch_bounds__(SCAN_BLOCK) void k_compact_count(const int32_t *st, const uint64_t *counts, uint64_t n,
                                                              uint64_t *part) {
    const uint64_t k = (uint64_t)blockIdx.x * SCAN_BLOCK + threadIdx.x;
    const int c = __syncthreads_count(handed_on(st, min(counts[0], n), k));
    if (threadIdx.x == 0) part[blockIdx.x] = (uint64_t)c;
}

__global__ __launch_bounds__(SCAN_BLOCK) void k_compact_write(const uint64_t *d_off, const uint32_t *d_len,
                                                              const int32_t *st, const uint64_t *counts, uint64_t n,
                                                              const uint64_t *part, uint64_t nb, uint64_t *f_off,
                                                              uint32_t *f_len, int64_t *frame_pair,
                                                              int64_t *n_frames) {
    __shared__ uint32_t wave_n[SCAN_BLOCK / 64];
    const uint64_t k = (uint64_t)blockIdx.x * SCAN_BLOCK + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const bool ok = handed_on(st, min(counts[0], n), k);
    const uint64_t bal = __ballot(ok);
    if (lane == 0) wave_n[w] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t before = (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
    for (uint32_t j = 0; j < w; ++j) before += wave_n[j];
    const uint64_t total = part[nb];
    if (ok) {
        const uint64_t r = part[blockIdx.x] + before;
        f_off[r] = d_off[k];
        f_len[r] = d_len[k];
        frame_pair[r] = (int64_t)k;
    }
    if (k < n && k >= total) {          // past the frames: empty, rejected by every later stage
        f_off[k] = 0;
        f_len[k] = 0;
        frame_pair[k] = -1;
    }
    if (k == 0) *n_frames = (int64_t)total;
}

// Packet.unpack's data (Packet.py:262-275): the token of packet i is
// pkt[pkt_off[i] + data_offset, + data_len) where unpack succeeded; an empty
// span at pkt_off[i] elsewhere (rejected by the decrypt as too short).
__global__ __launch_bounds__(256) void k_token_spans(const rt_packet_fields *f, const uint64_t *pkt_off, uint32_t n,
                                                     uint64_t *tok_off, uint32_t *tok_len) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t *r = (const uint32_t *)(f + i);       // ok in byte 0, data_offset / data_len in words 3 / 4
    const bool ok = (r[0] & 0xFFu) == 1u;
    tok_off[i] = pkt_off[i] + (ok ? r[3] : 0u);
    tok_len[i] = ok ? r[4] : 0u;
}

// --------------------------------------------------------- packet header --

// SHA-256 over  first || src[0..len): the full 64-B blocks from 16-B loads
// at src - 1 (that byte is readable: the packet's hop count or the transport
// id's last byte) with `first` put in front, the last block(s) byte by byte.
__device__ void sha_prefixed(uint8_t first, const uint8_t *src, uint32_t len, uint32_t out[8]) {
    uint32_t h[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) h[k] = SHA_IV[k];
    const uint32_t m = len + 1u;
    const uint64_t bits = (uint64_t)m * 8u;
    const uint32_t nfull = m / 64u;
    for (uint32_t b = 0; b < nfull; ++b) {
        const uint8_t *B = src - 1 + 64ull * b;
        uint32_t w[16];
        sha_units(w, ld16(B), ld16(B + 16), ld16(B + 32), ld16(B + 48));
        if (b == 0) w[0] = (w[0] & 0x00FFFFFFu) | ((uint32_t)first << 24);
        sha256_compress(h, w);
    }
    const uint32_t r = m - 64u * nfull;                 // 0..63 message bytes left
    const uint32_t nblk = (r + 8u) / 64u + 1u;
    for (uint32_t bb = 0; bb < nblk; ++bb) {
        uint32_t w[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            uint32_t v = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t q = 64u * (nfull + bb) + 4u * k + j;
                const uint32_t byte = q == 0 ? first : (q < m ? src[q - 1] : (q == m ? 0x80u : 0u));
                v = (v << 8) | byte;
            }
            w[k] = v;
        }
        if (bb + 1 == nblk) {
            w[14] = (uint32_t)(bits >> 32);
            w[15] = (uint32_t)bits;
        }
        sha256_compress(h, w);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) out[k] = h[k];
}

__global__ __launch_bounds__(256) void k_unpack(const uint8_t *pkt, const uint64_t *off, const uint32_t *len,
                                                rt_packet_fields *out, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t *raw = pkt + off[i];
    const uint32_t L = len[i];
    rt_packet_fields f;
    __builtin_memset(&f, 0, sizeof(f));
    if (L >= 2) {
        f.flags = raw[0];
        f.hops = raw[1];
        f.header_type = (f.flags >> 6) & 1u;
        f.context_flag = (f.flags >> 5) & 1u;
        f.transport_type = (f.flags >> 4) & 1u;
        f.destination_type = (f.flags >> 2) & 3u;
        f.packet_type = f.flags & 3u;
        const uint32_t ctx_at = f.header_type ? 2u * DST_LEN + 2u : DST_LEN + 2u;
        // hops < PATHFINDER_M (Packet.py:242-243); ord() of the context byte needs it present
        if (f.hops < PATHFINDER_M && L > ctx_at) {
            f.ok = 1;
            f.context = raw[ctx_at];
            f.data_offset = ctx_at + 1u;
            f.data_len = L - f.data_offset;
            const uint8_t *dst = raw + (f.header_type ? 2u + DST_LEN : 2u);
            for (int k = 0; k < 16; ++k) f.destination_hash[k] = dst[k];
            if (f.header_type)
                for (int k = 0; k < 16; ++k) f.transport_id[k] = raw[2 + k];
            // get_hashable_part: flags & 0x0F || raw[2:] (header 1) or raw[18:] (header 2)
            const uint32_t from = f.header_type ? DST_LEN + 2u : 2u;
            uint32_t d[8];
            sha_prefixed(f.flags & 0x0Fu, raw + from, L - from, d);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                f.packet_hash[4 * k] = d[k] >> 24; f.packet_hash[4 * k + 1] = d[k] >> 16;
                f.packet_hash[4 * k + 2] = d[k] >> 8; f.packet_hash[4 * k + 3] = d[k];
            }
        }
    }
    out[i] = f;
}

// Header bytes from registers: the 16-B fields are loaded whole and shifted by
// two bytes across words (v_alignbit), so a HEADER_1 is one 16-B store plus
// 2 + 1 bytes (HEADER_2: two 16-B stores plus 2 + 1); storing byte by byte
// took 217 us for 2^20 headers (profiles/r03ab_node/).  The bytes after the
// header (the packet's token, already in place) are not touched.
__device__ __forceinline__ u32x4 shift_in2(uint32_t lo2, u32x4 d) {
    // lo2 (2 bytes) || d[0..13]
    return u32x4{(lo2 & 0xFFFFu) | (d.x << 16), __builtin_amdgcn_alignbit(d.y, d.x, 16),
                 __builtin_amdgcn_alignbit(d.z, d.y, 16), __builtin_amdgcn_alignbit(d.w, d.z, 16)};
}
__global__ __launch_bounds__(256) void k_pack_headers(PackArgs a) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    uint8_t *o = a.out + a.out_off[i];
    const uint32_t fh = (uint32_t)a.flags[i] | (a.hops ? (uint32_t)a.hops[i] << 8 : 0u);
    const u32x4 dh = ld16(a.destination_hash + 16ull * i);
    u32x4 last = dh;                                    // the field whose bytes 14, 15 end the header
    if (a.transport_id) {
        const u32x4 tid = ld16(a.transport_id + 16ull * i);
        st16(o, shift_in2(fh, tid));
        st16(o + 16, shift_in2(tid.w >> 16, dh));
        o += 32;
    } else {
        st16(o, shift_in2(fh, dh));
        o += 16;
    }
    const uint16_t t2 = (uint16_t)(last.w >> 16);
    __builtin_memcpy(o, &t2, 2);
    o[2] = a.context[i];
}

}  // namespace

// ------------------------------------------------------------- launchers --

uint64_t scan_workspace_bytes(uint64_t n) { return 8ull * ((n + SCAN_BLOCK - 1) / SCAN_BLOCK + 1); }

// out[i] = sum(in[0..i)); *total (device) = sum(in)
static hipError_t launch_scan(const uint64_t *in, uint64_t *out, uint64_t n, uint64_t *part, uint64_t *total,
                              hipStream_t s) {
    const uint64_t nb = (n + SCAN_BLOCK - 1) / SCAN_BLOCK;
    if (nb == 0) return hipSuccess;
    hipLaunchKernelGGL(k_scan_block, dim3((unsigned)nb), dim3(SCAN_BLOCK), 0, s, in, out, part, n);
    hipLaunchKernelGGL(k_scan_parts, dim3(1), dim3(SCAN_BLOCK), 0, s, part, nb);
    hipLaunchKernelGGL(k_scan_add, dim3((unsigned)nb), dim3(SCAN_BLOCK), 0, s, out, part, n, total);
    return hipGetLastError();
}

uint64_t hdlc_frame_workspace_bytes(uint32_t n) { return 8ull * n + scan_workspace_bytes(n) + 64; }

hipError_t launch_hdlc_frame(const uint8_t *pkt, const uint64_t *off, const uint32_t *len, uint32_t n, uint8_t *out,
                             uint64_t *frame_off, void *ws, hipStream_t s) {
    if (n == 0) return hipSuccess;
    uint64_t *flen = (uint64_t *)ws;
    uint64_t *part = flen + n;
    // one DPP row per packet: 16 packets per 256-thread workgroup, grid-stride
    const unsigned g = (unsigned)min((uint64_t)(n + 15) / 16, (uint64_t)WAVE_GRID);
    hipLaunchKernelGGL(k_hdlc_count, dim3(g), dim3(256), 0, s, pkt, off, len, flen, n);
    hipError_t e = launch_scan(flen, frame_off, n, part, frame_off + n, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_hdlc_write, dim3(g), dim3(256), 0, s, pkt, off, len, frame_off, out, n);
    return hipGetLastError();
}

uint64_t hdlc_deframe_workspace_bytes(uint64_t len) {
    const uint64_t chunks = (len + FLAG_CHUNK - 1) / FLAG_CHUNK;
    return 8ull * chunks * 2 + scan_workspace_bytes(chunks) + 8ull * (len + 1) + 64 + 2ull * FLAG_CHUNK * chunks;
}

hipError_t launch_hdlc_deframe(const uint8_t *buf, uint64_t len, uint32_t hw_mtu, uint32_t ifac_size, uint8_t *out,
                               uint64_t *frame_off, uint32_t *frame_len, int32_t *status, uint64_t *counts,
                               uint64_t max_pairs, void *ws, hipStream_t s, uint32_t line_phase) {
    const uint64_t chunks = (len + FLAG_CHUNK - 1) / FLAG_CHUNK;
    uint64_t *cnt = (uint64_t *)ws;
    uint64_t *cnt_off = cnt + chunks;
    uint64_t *part = cnt_off + chunks;
    // part[nb] receives the scanned total (k_scan_parts): the flag count
    uint64_t *nflags = part + (chunks + SCAN_BLOCK - 1) / SCAN_BLOCK;
    uint64_t *pos = nflags + 2;
    uint16_t *loc = (uint16_t *)(pos + len + 1);         // chunk-local positions (k_flag_local)
    hipError_t e;
    if (!chunks && (e = hipMemsetAsync(nflags, 0, 8, s)) != hipSuccess) return e;   // else k_scan_parts writes it
    if (chunks) {
        hipLaunchKernelGGL(k_flag_local, dim3((unsigned)chunks), dim3(256), 0, s, buf, len, cnt, loc);
        // chunk counts scanned within blocks, then the block totals (part[nb] = the flag count);
        // the gather adds the two
        const uint64_t nb = (chunks + SCAN_BLOCK - 1) / SCAN_BLOCK;
        hipLaunchKernelGGL(k_scan_block, dim3((unsigned)nb), dim3(SCAN_BLOCK), 0, s, cnt, cnt_off, part, chunks);
        hipLaunchKernelGGL(k_scan_parts, dim3(1), dim3(SCAN_BLOCK), 0, s, part, nb);
        hipLaunchKernelGGL(k_flag_gather, dim3((unsigned)((chunks + 3) / 4)), dim3(256), 0, s, cnt, cnt_off, part, loc,
                           chunks, pos);
    }
    // the pair count lives on the device: a grid-stride kernel sized by the caller's capacity
    if (max_pairs) {
        const uint64_t g = min((max_pairs + 15) / 16, (uint64_t)WAVE_GRID);   // one DPP row per frame
        hipLaunchKernelGGL(k_hdlc_unescape, dim3((unsigned)g), dim3(256), 0, s, buf, len, pos, nflags, max_pairs,
                           hw_mtu, ifac_size, out, frame_off, frame_len, status, counts, line_phase);
    } else {
        hipLaunchKernelGGL(k_deframe_counts, dim3(1), dim3(1), 0, s, nflags, pos, len, hw_mtu, counts);
    }
    return hipGetLastError();
}

hipError_t launch_ifac(const IfacArgs &a, bool mask, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    const unsigned g = (a.n + 255) / 256;
    if (mask)
        hipLaunchKernelGGL(k_ifac<true>, dim3(g), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(k_ifac<false>, dim3(g), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_unpack(const uint8_t *pkt, const uint64_t *off, const uint32_t *len, void *fields, uint32_t n,
                         hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_unpack, dim3((n + 255) / 256), dim3(256), 0, s, pkt, off, len, (rt_packet_fields *)fields, n);
    return hipGetLastError();
}

uint64_t frames_compact_workspace_bytes(uint64_t max_pairs) { return scan_workspace_bytes(max_pairs); }

hipError_t launch_frames_compact(const uint64_t *d_off, const uint32_t *d_len, const int32_t *st,
                                 const uint64_t *counts, uint64_t max_pairs, uint64_t *f_off, uint32_t *f_len,
                                 int64_t *frame_pair, int64_t *n_frames, void *ws, hipStream_t s) {
    if (max_pairs == 0) return hipMemsetAsync(n_frames, 0, 8, s);
    const uint64_t nb = (max_pairs + SCAN_BLOCK - 1) / SCAN_BLOCK;
    uint64_t *part = (uint64_t *)ws;
    hipLaunchKernelGGL(k_compact_count, dim3((unsigned)nb), dim3(SCAN_BLOCK), 0, s, st, counts, max_pairs, part);
    hipLaunchKernelGGL(k_scan_parts, dim3(1), dim3(SCAN_BLOCK), 0, s, part, nb);
    hipLaunchKernelGGL(k_compact_write, dim3((unsigned)nb), dim3(SCAN_BLOCK), 0, s, d_off, d_len, st, counts,
                       max_pairs, part, nb, f_off, f_len, frame_pair, n_frames);
    return hipGetLastError();
}

hipError_t launch_token_spans(const void *fields, const uint64_t *pkt_off, uint32_t n, uint64_t *tok_off,
                              uint32_t *tok_len, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_token_spans, dim3((n + 255) / 256), dim3(256), 0, s, (const rt_packet_fields *)fields,
                       pkt_off, n, tok_off, tok_len);
    return hipGetLastError();
}

hipError_t launch_pack_headers(const PackArgs &a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_pack_headers, dim3((a.n + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace rnstok
