// token_kernels.hip — HIP kernels for the encrypted-token path on gfx950.
//
//   k_key_setup  : per key, AES key expansion (aes256.py:146-175 / aes128.py),
//                  equivalent-inverse-cipher schedule, HMAC ipad/opad midstates
//                  (HMAC.py:73-84).  One lane per key.
//   k_encrypt    : Token.encrypt (Token.py:87-97) — one packet per lane:
//                  PKCS7 pad, AES-CBC (serial chain in VGPRs, T-tables in LDS),
//                  HMAC-SHA256 over iv||ct interleaved with the chain (one
//                  SHA-256 compression per four cipher blocks).
//   k_decrypt    : Token.verify_hmac + Token.decrypt (Token.py:77-84,100-114) —
//                  one token per lane: HMAC verify and CBC decrypt in one pass
//                  over the token, lenient PKCS7 unpad (PKCS7.py:42-48).
//
// Launch shape: one 1024-thread (single key) or 768/512-thread (per-packet keys)
// workgroup per CU, persistent over the batch; the LDS table image is built
// once per workgroup.  See DESIGN.md.
#include "keysetup_device.h"
#include "token_device.h"
#include "token_launch.h"
#include "../../include/rnstok.h"

namespace rnstok {

// Workgroup sizes: one workgroup per CU (the LDS table image is 128/160 KiB).
// Packed rows: 16-B units at a 560-B row stride share 128-B lines between
// consecutive quads, and one quad apart the line has left L2 (profiles/r04o,
// r04p, r04q, one-process A/Bs at c2 / 1500 B / packed):
#ifndef RNSTOK_ENC_PAIR              // split encrypt, plaintext quads loaded in pairs: fetch -13 %, time -0.5 %
#define RNSTOK_ENC_PAIR 1
#endif
// (split encrypt, token quads stored in pairs: writes -22 %, time +2.2 %: not adopted, r04q)
#ifndef RNSTOK_SPLIT_TILE            // experiment: packed split encrypt reads 64-packet plaintext tiles
#define RNSTOK_SPLIT_TILE 0
#endif
#ifndef RNSTOK_DEC_TAG_EARLY         // decrypt: tag units loaded before the quad loop
#define RNSTOK_DEC_TAG_EARLY 1
#endif
#ifndef RNSTOK_DEC_PAIR              // decrypt, one key, token quads loaded in pairs: fetch -21 %, time -1.6 %
#define RNSTOK_DEC_PAIR 1
#endif
// Split encrypt, packed rows: the ciphertext units of a 64-B sector that a quad
// shares with the next quad are held and stored with the next quad's, so every
// sector leaves in one burst of stores (fabric write requests 18.3 M -> 12.8 M
// per c2 launch, the count of the same tokens with their ciphertext on lines).
// The chip then holds a higher clock: whole-bench A/Bs (each variant its own
// sustained run) c2 +2.2 % (2.20 -> 2.25 GHz, cycles equal), per-packet keys
// c3 encrypt -2.9 %, c5's encrypt half -4.7 % (profiles/r06_clock_ab/).  An A/B
// that interleaves the variants launch by launch shares one clock between
// them and showed +1.3 %.
#ifndef RNSTOK_ENC_ST_SECTOR
#define RNSTOK_ENC_ST_SECTOR 1
#endif
#ifndef RNSTOK_ENC_ST_SECTOR_PERKEY  // per-packet keys: with single plaintext quads (next line) 5 VGPRs
#define RNSTOK_ENC_ST_SECTOR_PERKEY 1  // spilled; with the paired loads 31
#endif
#ifndef RNSTOK_ENC_PAIR_PERKEY       // per-packet keys: plaintext quads loaded in pairs (off: the
#define RNSTOK_ENC_PAIR_PERKEY 0     // registers go to the held sector units)
#endif
#ifndef RNSTOK_SPLIT_DYN              // split encrypt: unevenly divided uniform batches from a counter
#define RNSTOK_SPLIT_DYN 1
#endif
#ifndef RNSTOK_SPLIT_DYN_MIN_LEN
#define RNSTOK_SPLIT_DYN_MIN_LEN 256u
#endif
#ifndef RNSTOK_DEC1024_MAX_TOKEN     // uniform tokens up to this length: the 1024-thread decrypt
#define RNSTOK_DEC1024_MAX_TOKEN 320u  // (plaintexts up to 271 B)
#endif
#ifndef RNSTOK_WG_ENC
#define RNSTOK_WG_ENC 1024      // single key: 4 waves/SIMD, 128 VGPRs
#endif
#ifndef RNSTOK_WG_DEC
#define RNSTOK_WG_DEC 768       // 3 waves/SIMD, no spills; with the chunk loop for c2's ragged
                                // 5.33 packets per lane: 2 % faster than 1024 (A/B, 30 rounds)
#endif
// per-packet keys: the round keys live in VGPRs, so fewer waves per SIMD
#ifndef RNSTOK_WG_PERKEY_ENC
#define RNSTOK_WG_PERKEY_ENC 768   // <= 168 VGPRs, 3 waves/SIMD
#endif
#ifndef RNSTOK_WG_PERKEY_DEC
#define RNSTOK_WG_PERKEY_DEC 768   // <= 168 VGPRs, 3 waves/SIMD (c3: 5.5 % faster than 512 threads
                                   // at 256 VGPRs, despite some spilling; needs the chunk loop's balance)
#endif
constexpr int WG_ENC = RNSTOK_WG_ENC, WG_DEC = RNSTOK_WG_DEC;
// Optional explicit occupancy target (waves per SIMD) for the single-key
// kernels, so the scheduler may spend registers on loads in flight.
#ifdef RNSTOK_WAVES_PER_EU
#define RT_OCC __attribute__((amdgpu_waves_per_eu(RNSTOK_WAVES_PER_EU, RNSTOK_WAVES_PER_EU)))
#else
#define RT_OCC
#endif
constexpr int WG_PERKEY_ENC = RNSTOK_WG_PERKEY_ENC, WG_PERKEY_DEC = RNSTOK_WG_PERKEY_DEC;

// ------------------------------------------------------------ LDS tables --

__device__ __forceinline__ uint32_t xt(uint32_t b) { return ((b << 1) ^ ((b & 0x80u) ? 0x1bu : 0u)) & 0xffu; }
__device__ __forceinline__ uint32_t gmul(uint32_t a, uint32_t b) {
    uint32_t p = 0;
    for (int i = 0; i < 8; ++i) {
        if (b & 1) p ^= a;
        a = xt(a);
        b >>= 1;
    }
    return p;
}
__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) { return n ? ((x << n) | (x >> (32 - n))) : x; }

// T0[x] = {02*S, 01*S, 01*S, 03*S} (bytes = rows 0..3 of the column word)
__device__ __forceinline__ uint32_t te0(const uint8_t *sbox, uint32_t x) {
    uint32_t s = sbox[x], s2 = xt(s);
    return s2 | (s << 8) | (s << 16) | ((s2 ^ s) << 24);
}
// Td0[x] = {0e*y, 09*y, 0d*y, 0b*y}, y = InvS[x]
__device__ __forceinline__ uint32_t td0(const uint8_t *inv, uint32_t x) {
    uint32_t y = inv[x];
    return gmul(y, 14) | (gmul(y, 9) << 8) | (gmul(y, 13) << 16) | (gmul(y, 11) << 24);
}

template <bool DEC>
__device__ void fill_tables(uint32_t *tab, const uint8_t *sbox, const uint8_t *inv) {
    // regions 0,1: 32768 dwords; dword d -> region d>>14, row (d>>6)&255,
    // table (d>>5)&1, replica d&31.  One unit = (row x, rotation t): its entry
    // is computed once and stored to its 32 replicas, the replica order
    // rotated by lane so each half-wave's stores hit 32 distinct banks.  (The
    // per-dword form recomputed Td0's GF multiplies 128 times per row and
    // cost ≈40 µs in a one-workgroup launch.)
    const uint32_t lane = threadIdx.x & 31u;
    for (uint32_t u = threadIdx.x; u < 1024u; u += blockDim.x) {
        const uint32_t x = u & 255u, t = u >> 8;
        const uint32_t v = rotl(DEC ? td0(inv, x) : te0(sbox, x), 8 * (int)t);
        uint32_t *row = tab + ((t >> 1) << 14) + (x << 6) + ((t & 1u) << 5);
#pragma unroll 8
        for (uint32_t j = 0; j < 32u; ++j) row[(j + lane) & 31u] = v;
    }
    if (DEC) {
        for (uint32_t x = threadIdx.x; x < 256u; x += blockDim.x) {
            const uint32_t v = (uint32_t)inv[x] * 0x01010101u;
            uint32_t *row = tab + 32768u + (x << 5);
#pragma unroll 8
            for (uint32_t j = 0; j < 32u; ++j) row[(j + lane) & 31u] = v;
        }
    }
    __syncthreads();
}

// --------------------------------------------------------------- layout --

struct Layout {
    const uint64_t *off;   // per-packet offsets, or null: i * stride
    uint64_t stride;
    const uint32_t *len;   // per-packet lengths, or null: uniform
    uint32_t uni;
    __device__ __forceinline__ uint64_t o(uint32_t i) const { return off ? off[i] : (uint64_t)i * stride; }
    __device__ __forceinline__ uint32_t l(uint32_t i) const { return len ? len[i] : uni; }
};

__device__ __forceinline__ uint64_t in_off(const uint64_t *off, uint64_t stride, uint32_t i) {
    return off ? off[i] : (uint64_t)i * stride;
}

template <int NR, bool PERKEY>
struct Keys {
    uint32_t rk[4 * (NR + 1)];
    __device__ __forceinline__ void load(const uint32_t *rec, int base) {
        if (PERKEY) {
#pragma unroll
            for (int i = 0; i < NR + 1; ++i) {
                u32x4 v = *(const u32x4 *)(rec + base + 4 * i);
                rk[4 * i] = v.x; rk[4 * i + 1] = v.y; rk[4 * i + 2] = v.z; rk[4 * i + 3] = v.w;
            }
        } else {
            // one key for the whole launch: keep the schedule in SGPRs (VOP3
            // operands), leaving the VGPR budget to the AES/SHA chains (a VALU
            // op with an SGPR operand issues at half rate, but the schedule in
            // VGPRs, whole or in part, measured slower: DESIGN.md §4.5)
#pragma unroll
            for (int i = 0; i < 4 * (NR + 1); ++i) rk[i] = __builtin_amdgcn_readfirstlane(rec[base + i]);
        }
    }
};

// Uniform 8-word load re-issued per packet (scalar cache hit) instead of
// being kept live in SGPRs across the packet loop.
__device__ __forceinline__ void load_uniform8(uint32_t d[8], const uint32_t *p) {
    asm volatile("" : "+s"(p));
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = __builtin_amdgcn_readfirstlane(p[i]);
}

__device__ __forceinline__ void load8(uint32_t d[8], const uint32_t *p) {
    u32x4 a = *(const u32x4 *)p, b = *(const u32x4 *)(p + 4);
    d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w; d[4] = b.x; d[5] = b.y; d[6] = b.z; d[7] = b.w;
}

// ---------------------------------------------------------- packet loop --
//
// One packet per lane.  Uniform batches use a static grid stride (every lane
// gets the same work).  Length-ordered batches (a.queue set, packets sorted
// by descending length) hand out 64-packet chunks from a global counter, one
// atomic per wave and chunk: the longest packets start first and the chunks
// that finish last are the shortest, so the CUs end together.  A static
// stride over the sorted order gave the first workgroup the longest packet of
// every pass (c5: 40 % more work than the average CU).
// The chunk counter (32 bits) may run up to n + 64 x the grid's waves.
constexpr uint32_t QUEUE_MAX_N = 0xF0000000u;
__device__ __forceinline__ uint32_t take_chunk(uint32_t *q) {
    uint32_t v = 0u;
    if ((threadIdx.x & 63u) == 0u) v = __hip_atomic_fetch_add(q, 64u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return __builtin_amdgcn_readlane(v, 0);
}
// Lane 0 carries the wave's smallest index, so it stays active until the
// whole wave leaves (lanes past n break out of the last chunk only).
// The index runs in 64 bits so that a batch near 2^32 packets cannot wrap
// it (the launchers use the chunk counter only below QUEUE_MAX_N).
#define RT_PACKET_LOOP(A, I)                                                                                 \
    for (uint64_t rt_base_ = (A).queue ? take_chunk((A).queue) : blockIdx.x * blockDim.x + (threadIdx.x & ~63u), \
                  rt_i_ = rt_base_ + (threadIdx.x & 63u);                                                     \
         rt_i_ < (A).n;                                                                                       \
         rt_base_ = (A).queue ? take_chunk((A).queue) : rt_base_ + (uint64_t)gridDim.x * blockDim.x,         \
                  rt_i_ = rt_base_ + (threadIdx.x & 63u))                                                     \
        if (const uint32_t I = (uint32_t)rt_i_; true)

// ------------------------------------------------------------ launch clock --
//
// rt_clock_stamps: each workgroup of a stamped launch adds its span in shader
// clock cycles (s_memtime) and in 100 MHz real-time ticks (s_memrealtime) to
// its kernel class's words: {sum of cycles, sum of ticks, workgroups, launches}.
// The sustained clock of the run is cycles / ticks x 100 MHz and the cycles per
// launch the mean workgroup span (one persistent workgroup per CU), measured
// in the run itself instead of read from a profile of another box.  The end
// stamp follows a workgroup barrier, so the span covers every wave; the
// uniform pointer keeps the branch (and the barrier) wave- and
// workgroup-uniform.  Off (null), it costs one scalar compare per launch.
struct LaunchClock {
    uint64_t c0 = 0, r0 = 0;
    __device__ __forceinline__ void start(const unsigned long long *acc) {
        if (acc) {
            c0 = __builtin_amdgcn_s_memtime();
            r0 = __builtin_amdgcn_s_memrealtime();
        }
    }
    __device__ __forceinline__ void finish(unsigned long long *acc) const {
        if (!acc) return;
        __syncthreads();
        if (threadIdx.x == 0u) {
            const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
            __hip_atomic_fetch_add(acc + 0, (unsigned long long)(c1 - c0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(acc + 1, (unsigned long long)(r1 - r0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(acc + 2, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (blockIdx.x == 0u) __hip_atomic_fetch_add(acc + 3, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
};

// PKCS7 pad block (PKCS7.py:35-39): r (< 16) payload bytes at p, then 16-r copies of 16-r.
__device__ __forceinline__ u32x4 pad_block(const uint8_t *p, uint32_t r) {
    uint32_t n = 16u - r, w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        uint32_t b = ((uint32_t)i < r) ? (uint32_t)p[i] : n;
        w[i >> 2] |= b << (8 * (i & 3));
    }
    u32x4 v = {w[0], w[1], w[2], w[3]};
    return v;
}

// --------------------------------------------------------------- encrypt --

// ILV: the unit-interleaved layout of rt_encrypt_interleaved (16-B unit u of
// packet p at 16*(u*n + p) in the plaintext and token buffers): every wave
// load/store instruction then covers 1 KiB of contiguous HBM instead of 64
// scattered 16-B pieces.  US is the distance between a
// packet's consecutive units.
template <int NR, bool PERKEY, bool ILV = false>
__global__ RT_OCC __launch_bounds__(PERKEY ? WG_PERKEY_ENC : WG_ENC) void k_encrypt(EncArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t tab_u32[];
    LaunchClock clk;
    clk.start(a.clk);
    fill_tables<false>(tab_u32, a.sbox, a.sbox + 256);
    const Lanes LN(threadIdx.x & 31u);

    Keys<NR, PERKEY> K;
    uint32_t ipad[8], opad[8];
    if (!PERKEY) K.load(a.rec, REC_ENC);
    const Layout in{a.pt_off, a.pt_stride, a.pt_len, a.uni_len};

    RT_PACKET_LOOP(a, i) {
        const uint32_t p = a.order ? a.order[i] : i;
        // the opad midstate is loaded after the quad loop, so it does not
        // hold registers through it
        const uint32_t *r = PERKEY ? a.rec + (uint64_t)a.key_idx[p] * REC_WORDS : a.rec;
        if (PERKEY) {
            K.load(r, REC_ENC);
            load8(ipad, r + REC_IPAD);
        } else {
            load_uniform8(ipad, a.rec + REC_IPAD);
        }
        const uint32_t L = in.l(p);
        const uint64_t US = ILV ? 16ull * a.n : 16ull;
        const uint8_t *P = ILV ? a.pt + 16ull * p : a.pt + in.o(p);
        uint8_t *O = ILV ? a.tok + 16ull * p : a.tok + (a.tok_off ? a.tok_off[p] : (uint64_t)p * a.tok_stride);
        const u32x4 iv = ld16(a.iv + 16ull * p);
        st16(O, iv);
        uint8_t *C = O + US;

        const uint32_t nfull = L >> 4, nq = nfull >> 2, tb = (nfull & 3u) + 1u;
        uint32_t h[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) h[i] = ipad[i];
        // One loop body serves every quad, the tail quad (tb blocks, the last
        // one carrying the PKCS7 pad; unused slots run on zeros and are not
        // stored) included; the SHA-256 compression of quad q-1's units rides
        // on quad q's AES chain (quad 0 has none and runs the chain alone).
        // hmac_finish runs the last 2-3 compressions through one
        // sha256_compress: ≈75 KB of code where a head/body/tail-specialised
        // loop took 150 KB (same speed on c2, measured; 2-7 % faster with
        // per-packet keys).
        {
            const u32x4 z = {0u, 0u, 0u, 0u};
            const uint32_t rem = L & 15u;
            u32x4 prev = iv, x[4], c[4];
            Sha256 S;                       // S.w: the pending SHA block (previous quad's units)
#pragma unroll
            for (int k = 0; k < 16; ++k) S.w[k] = 0u;
            // Quad 0 is peeled: the AES chain alone (no SHA block yet), so
            // the loop carries its SHA rounds unconditionally (a loop that
            // branched on q == 0 was unswitched by the compiler into one body
            // with a scalar branch around every SHA round: 1.8 % slower, A/B).
            auto load_quad = [&](uint32_t q) {
                if (q < nq) {
                    x[0] = ld16(P); x[1] = ld16(P + US); x[2] = ld16(P + 2 * US); x[3] = ld16(P + 3 * US);
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        x[j] = (uint32_t)j + 1u < tb ? ld16(P + US * j)
                                                     : ((uint32_t)j + 1u == tb ? pad_block(P + US * j, rem) : z);
                }
            };
            auto store_quad = [&](uint32_t q) {
                const uint32_t nst = q < nq ? 4u : tb;
                st16(C, c[0]);
                if (nst > 1u) st16(C + US, c[1]);
                if (nst > 2u) st16(C + 2 * US, c[2]);
                if (nst > 3u) st16(C + 3 * US, c[3]);
            };
            load_quad(0u);
            enc_quad<NR, false>(c, x, prev, K.rk, LN, S);
            store_quad(0u);
            sha_units(S.w, prev, c[0], c[1], c[2]);
            prev = c[3];
            P += 4 * US; C += 4 * US;
#pragma nounroll
            for (uint32_t q = 1; q <= nq; ++q) {
                load_quad(q);
                S.start(h);
                enc_quad<NR, true>(c, x, prev, K.rk, LN, S);
                // The SHA rounds' results are consumed here, in the AES
                // chain's block: otherwise the compiler sinks the rounds past
                // the stores below and the two chains run back to back.
#pragma unroll
                for (int k = 0; k < 8; ++k) asm volatile("" ::"v"(S.v[k]));
#pragma unroll
                for (int k = 0; k < 8; ++k) h[k] += S.v[k];
                store_quad(q);
                sha_units(S.w, prev, c[0], c[1], c[2]);
                prev = c[3];
                P += 4 * US; C += 4 * US;
            }
            // S.w: units u0..u3 of the tail quad (u0 = the block before it),
            // prev = u4; tu = tb + 1 units are left for the inner hash: a full
            // block u0..u3 when tu >= 4, then the final padded block.
            const uint32_t tu = tb + 1u;
            uint32_t u4[16], fin[16];
            sha_units(u4, prev, z, z, z);
#pragma unroll
            for (int k = 0; k < 16; ++k) u4[k] = tu >= 4u ? u4[k] : S.w[k];
            sha_final_block(fin, u4, tu >= 4u ? tu - 4u : tu, (uint64_t)(64u + 16u + 16u * (nfull + 1u)) * 8u);
            if (PERKEY)
                load8(opad, r + REC_OPAD);
            else
                load_uniform8(opad, a.rec + REC_OPAD);
            hmac_finish(h, tu >= 4u ? 0u : 1u, S.w, fin, opad);
            uint8_t *T = O + US * (nfull + 2u);
            st16(T, u32x4{bswap(h[0]), bswap(h[1]), bswap(h[2]), bswap(h[3])});
            st16(T + US, u32x4{bswap(h[4]), bswap(h[5]), bswap(h[6]), bswap(h[7])});
        }
    }
    clk.finish(a.clk);
}

// ----------------------------------------------------- encrypt, split roles --
//
// The same work as k_encrypt with the two chains on waves of their own
// (VERDICT r03 next #2): waves 0..7 of the 1024-thread workgroup (two per
// SIMD; wave w sits on SIMD w % 4) run the CBC chains of 64 packets each, one
// per lane, and store the ciphertext; waves 8..15 (two per SIMD) hash it,
// wave 8+k the packets of AES wave k on the same SIMD.  In register-only
// loops this mix issues 19 % fewer SIMD-cycles per (AES quad + SHA-256
// compression) than one wave carrying both chains (tools/floor_probe.hip
// core_split8 10 188 vs core_enc 12 583, profiles/r04_split/r04b_floor_split.txt).
//
// Hand-over, two instances (A/B in one process against k_encrypt, tokens
// identical, profiles/r04_split/r04f_three_way_ab.txt, r04h_enc_dec_split_ab.txt):
// * packed rows (RB = false): an LDS ring after the 128 KiB table image, one
//   slot of one quad per lane (4 KiB per AES wave, 16-B unit j of lane l at
//   1024 j + 16 l: conflict-free ds_write_b128 / ds_read_b128), which fills
//   the CU's 160 KiB.  The two hand-over counters of each wave pair live in
//   lane 0's first unit, so lane 0's quad goes another way: the hashing wave's
//   lane 0 reads it back from the token buffer.  500 B: 0.857 vs 0.891 ms
//   (-3.8 %) and 0.839 vs 0.886 (-5.3 %) on two boxes; 1500 B -2.5 / -3.1 %.
//   Reading every lane's quad back from the token rows instead (a second
//   scattered 16-B pattern) is 1.6 % slower at 500 B.
// * interleaved (RB = true): no ring, every hashing lane reads its quad back
//   from the token buffer (coalesced 1-KiB reads, L2 hits, no LDS instruction
//   taken from the lookups' pipe): 0.743 vs 0.814 ms (-8.8 %), 1500 B -9.6 %;
//   the LDS ring there: -3.7 %.  (A staging ring in global memory instead of
//   LDS: -2.4 % rows, -2.8 % interleaved: 4 more stores per quad, ring lines
//   leaving L2; profiles/r04_split/r04d_global_stage_ab.txt.)
// AES wave k stores quad q's ciphertext, writes it to its slot and publishes
// its count of quads with a workgroup-scope release; hashing wave 8+k waits
// for that count (s_sleep), reads the slot after an acquire and publishes its
// own count, which the AES wave checks before it overwrites the slot.  One
// slot is enough: the hashing wave takes a quad as soon as it is there unless
// it is finishing a packet (3 compressions), which is shorter than two AES
// quads.  Every wave leaves after the same batches, so the grid always
// drains.  Uniform lengths (rows at a stride, or ILV), one key or per-packet
// keys (PERKEY: each AES lane loads its packet's round keys, each hashing lane
// its ipad/opad midstates, from the 544-B key records; 128 VGPRs, 2 spilled
// on rows).
#ifndef RNSTOK_SPLIT_AES_WAVES       // AES waves (= hashing waves) per workgroup (experiment knob)
#define RNSTOK_SPLIT_AES_WAVES 8
#endif
constexpr uint32_t SPLIT_AES_WAVES = RNSTOK_SPLIT_AES_WAVES, SPLIT_THREADS = 128u * RNSTOK_SPLIT_AES_WAVES;
constexpr uint32_t SPLIT_RING = LDS_ENC_BYTES;                    // 8 x 4 KiB
constexpr uint32_t LDS_ENC_SPLIT_BYTES = SPLIT_RING + SPLIT_AES_WAVES * 4096u;
static_assert(LDS_ENC_SPLIT_BYTES <= 160u * 1024u, "LDS");

// Wave maximum of a per-lane value (sorted chunks: lane 0 already holds it).
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = (uint32_t)__shfl_xor((int)v, d, 64);
        v = o > v ? o : v;
    }
    return v;
}

// GEN: packed batches (per-packet lengths and offsets, a length order and the
// chunk counter of RT_F_SORT_BY_LENGTH), the shape of c5's encrypt half.  The
// AES wave takes each 64-packet chunk (from the counter, or its static share)
// and hands the chunk's first index to the hashing wave in the slot's lane-0
// unit with the chunk's first quad; both run the chunk to its longest packet
// (a length-ordered chunk is nearly uniform), each lane stopping at its own
// last quad.  A chunk index past the batch tells the hashing wave to leave.
#ifdef RNSTOK_SPLIT_PROBE
// timing probe (probe builds only): per role, cycles spent waiting on the
// other role, waits entered, cycles from the table fill to the end
__device__ unsigned long long g_split_probe[8];
#define SPLIT_PROBE(x) x
#else
#define SPLIT_PROBE(x)
#endif
template <int NR, bool ILV = false, bool RB = ILV, bool PERKEY = false, bool GEN = false>
__global__ __launch_bounds__(SPLIT_THREADS) void k_encrypt_split(EncArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t tab_u32[];
    typedef __attribute__((address_space(3))) uint32_t lds_u32;
    typedef __attribute__((address_space(3))) u32x4 lds_q;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const bool aes = wave < SPLIT_AES_WAVES;
    const uint32_t pair = aes ? wave : wave - SPLIT_AES_WAVES;
    const uint32_t slot = SPLIT_RING + 4096u * pair;
    lds_u32 *produced = (lds_u32 *)(uintptr_t)slot, *consumed = (lds_u32 *)(uintptr_t)(slot + 4u);
    lds_u32 *chunk_at = (lds_u32 *)(uintptr_t)(slot + 8u);
    LaunchClock clk;
    clk.start(a.clk);
    if (aes && lane < 3u) ((lds_u32 *)(uintptr_t)slot)[lane] = 0u;   // before the barrier
    fill_tables<false>(tab_u32, a.sbox, a.sbox + 256);     // ends with the workgroup barrier
    SPLIT_PROBE(uint64_t pr_wait = 0; uint64_t pr_n = 0; const uint64_t pr_t0 = clock64();)

    const uint64_t US = ILV ? 16ull * a.n : 16ull;
    const uint32_t n_batches = (a.n + 63u) >> 6;
    const uint32_t first = blockIdx.x * SPLIT_AES_WAVES + pair, stride = gridDim.x * SPLIT_AES_WAVES;
    lds_q *mine = (lds_q *)(uintptr_t)(slot + 16u * lane);     // unit j at mine[64 j]
    const u32x4 z = {0u, 0u, 0u, 0u};
    uint32_t count = 0;                                    // quads handed over so far (both sides)
    // packet i of the batch: plaintext / token offsets, length
    auto pt_at = [&](uint32_t p) -> const uint8_t * {
        return ILV ? a.pt + 16ull * p : a.pt + (GEN && a.pt_off ? a.pt_off[p] : (uint64_t)p * a.pt_stride);
    };
    auto tok_at = [&](uint32_t p) -> uint8_t * {
        return ILV ? a.tok + 16ull * p : a.tok + (GEN && a.tok_off ? a.tok_off[p] : (uint64_t)p * a.tok_stride);
    };
    if (aes) {
        const Lanes LN(threadIdx.x & 31u);
        Keys<NR, PERKEY> K;
        if (!PERKEY) K.load(a.rec, REC_ENC);
        Sha256 S;                                          // unused: enc_quad<NR, false> hashes nothing
        uint32_t b = first;
        for (;;) {
            uint64_t base;
            if (GEN && a.queue) {
                base = take_chunk(a.queue);
            } else {
                base = 64ull * b;
                b += stride;
            }
            if (base >= a.n) {
                if (GEN) {             // tell the hashing wave (it cannot know the counter's end)
                    if (count)
                        while (__hip_atomic_load(consumed, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < count)
                            __builtin_amdgcn_s_sleep(1);
                    ++count;
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    if (lane == 0u) {
                        *chunk_at = 0xFFFFFFFFu;
                        __hip_atomic_store(produced, count, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
                break;
            }
            const uint32_t i = (uint32_t)base + lane;
            const bool valid = i < a.n;
            const uint32_t p = valid ? (GEN && a.order ? a.order[i] : i) : 0u;
            const uint32_t L = GEN && a.pt_len ? (valid ? a.pt_len[p] : 0u) : a.uni_len;
            const uint32_t nfull = L >> 4, nq = nfull >> 2, tb = (nfull & 3u) + 1u, rem = L & 15u;
            const uint32_t wq = GEN ? wave_max(valid ? nq : 0u) : nq;
            if (PERKEY) K.load(a.rec + (uint64_t)a.key_idx[p] * REC_WORDS, REC_ENC);
            const uint8_t *P = pt_at(p);
            uint8_t *O = tok_at(p);
            u32x4 prev = valid ? ld16(a.iv + 16ull * p) : z;
            uint8_t *C = O + US;
            // RNSTOK_ENC_ST_SECTOR (experiment): the ciphertext units of a 64-B
            // sector that a quad shares with the next are stored together with
            // the next quad's, so every sector is written by back-to-back stores
            // (sg: the sector phase of the lane's ciphertext start, in units)
            constexpr bool SECT = !ILV && (PERKEY ? RNSTOK_ENC_ST_SECTOR_PERKEY : RNSTOK_ENC_ST_SECTOR);
            // (lane 0 stores at once: its hashing lane reads the quad back from the token buffer)
            const uint32_t sg = SECT && lane ? ((uint32_t)(uintptr_t)C >> 4) & 3u : 0u;
            u32x4 cp1 = z, cp2 = z;                        // the previous quad's units 1, 2 (unit 3: prev)
            if (valid && (!SECT || sg == 0u)) st16(O, prev);
            // (experiment, RNSTOK_SPLIT_TILE: packed batches whose plaintexts a
            // gather pass laid out as 64-packet tiles, unit u of lane l at
            // pt_off + 1024 u; tokens stay byte strings)
            const uint64_t USP = GEN && RNSTOK_SPLIT_TILE ? 1024ull : US;
            // packed rows: full quads loaded in line-sharing pairs (k_decrypt)
            constexpr bool PAIR = (PERKEY ? RNSTOK_ENC_PAIR_PERKEY : RNSTOK_ENC_PAIR) && !ILV;
            u32x4 nx[4];
            for (uint32_t q = 0; q <= wq; ++q) {
                u32x4 x[4], c[4];
                const bool act = valid && q <= nq;
                if (PAIR && (q & 1u) && q < nq) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) x[j] = nx[j];
                } else if (q < nq) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) x[j] = valid ? ld16(P + USP * j) : z;
                    if (PAIR && q + 1u < nq) {
#pragma unroll
                        for (int j = 0; j < 4; ++j) nx[j] = valid ? ld16(P + USP * (4 + j)) : z;
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        x[j] = !act ? z
                                    : ((uint32_t)j + 1u < tb ? ld16(P + USP * j)
                                                             : ((uint32_t)j + 1u == tb ? pad_block(P + USP * j, rem) : z));
                }
                enc_quad<NR, false>(c, x, prev, K.rk, LN, S);
                const uint32_t nst = q < nq ? 4u : tb;
                if (SECT) {
                    if (act) {
                        if (q == 0u) {
                            if (sg != 0u) st16(C - US, prev);            // the IV, with its sector's units
                        } else {                                         // the previous quad's held units
                            if (sg == 3u) st16(C - 3 * US, cp1);
                            if (sg >= 2u) st16(C - 2 * US, cp2);
                            if (sg >= 1u) st16(C - US, prev);
                        }
                        const uint32_t now = q == nq ? nst : (4u - sg < nst ? 4u - sg : nst);
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            if ((uint32_t)j < now) st16(C + US * j, c[j]);
                    }
                    cp1 = c[1];
                    cp2 = c[2];
                } else if (act) {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if ((uint32_t)j < nst) st16(C + US * j, c[j]);
                }
                prev = c[3];
                P += 4 * USP;
                C += 4 * US;
                // the slot is free once the hashing wave has taken every earlier quad
                if (!RB && count) {
                    SPLIT_PROBE(const uint64_t pw = clock64(); bool pwt = false;)
                    while (__hip_atomic_load(consumed, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < count) {
                        SPLIT_PROBE(pwt = true;)
                        __builtin_amdgcn_s_sleep(1);
                    }
                    SPLIT_PROBE(if (pwt) { pr_wait += clock64() - pw; ++pr_n; })
                }
                if (!RB && lane) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) mine[64 * j] = c[j];
                }
                ++count;
                // lane 0's quad (read back from the token buffer) and the
                // slot's writes before the count the hashing wave polls: every
                // lane releases its own writes, lane 0 publishes the count
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (lane == 0u) {
                    if (GEN && q == 0u) *chunk_at = (uint32_t)base;
                    __hip_atomic_store(produced, count, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
        }
    } else {
        uint32_t b = first;
        for (;;) {
            uint64_t base;
            if (GEN) {
                while (__hip_atomic_load(produced, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < count + 1u)
                    __builtin_amdgcn_s_sleep(1);
                const uint32_t c0 = __builtin_amdgcn_readfirstlane(*chunk_at);
                if (c0 == 0xFFFFFFFFu) break;
                base = c0;
            } else {
                if (b >= n_batches) break;
                base = 64ull * b;
                b += stride;
            }
            const uint32_t i = (uint32_t)base + lane;
            const bool valid = i < a.n;
            const uint32_t p = valid ? (GEN && a.order ? a.order[i] : i) : 0u;
            const uint32_t L = GEN && a.pt_len ? (valid ? a.pt_len[p] : 0u) : a.uni_len;
            const uint32_t nfull = L >> 4, nq = nfull >> 2, tb = (nfull & 3u) + 1u;
            const uint32_t wq = GEN ? wave_max(valid ? nq : 0u) : nq;
            uint8_t *O = tok_at(p);
            const uint8_t *C = O + US;
            uint32_t h[8];
            const uint32_t *r = PERKEY ? a.rec + (uint64_t)a.key_idx[p] * REC_WORDS : a.rec;
            if (PERKEY)
                load8(h, r + REC_IPAD);
            else
                load_uniform8(h, a.rec + REC_IPAD);
            u32x4 up = valid ? ld16(a.iv + 16ull * p) : z;      // the unit before the quad (IV first)
            uint32_t w[16];
            for (uint32_t q = 0; q <= wq; ++q) {
                SPLIT_PROBE(const uint64_t pw = clock64(); bool pwt = false;)
                while (__hip_atomic_load(produced, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < count + 1u) {
                    SPLIT_PROBE(pwt = true;)
                    __builtin_amdgcn_s_sleep(1);
                }
                SPLIT_PROBE(if (pwt) { pr_wait += clock64() - pw; ++pr_n; })
                const uint32_t nst = q < nq ? 4u : tb;
                const bool act = valid && q <= nq;
                u32x4 c[4];
                if (!RB && lane) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) c[j] = mine[64 * j];
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j) c[j] = (act && (uint32_t)j < nst) ? ld16(C + US * j) : z;
                }
                ++count;
                // the slot's reads (every lane's) complete before the AES wave
                // may overwrite it
                if (!RB) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    if (lane == 0u)
                        __hip_atomic_store(consumed, count, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                C += 4 * US;
                if (!GEN || q <= nq) {
                    sha_units(w, up, c[0], c[1], c[2]);
                    if (q < nq) sha256_compress(h, w);
                    up = c[3];
                }
            }
            // w: units u0..u3 of the tail quad, up = u4 (units past the
            // packet's own are not hashed); tu = tb + 1 units are left for the
            // inner hash (as k_encrypt's tail)
            const uint32_t tu = tb + 1u;
            uint32_t u4[16], fin[16], opad[8];
            sha_units(u4, up, z, z, z);
#pragma unroll
            for (int k = 0; k < 16; ++k) u4[k] = tu >= 4u ? u4[k] : w[k];
            sha_final_block(fin, u4, tu >= 4u ? tu - 4u : tu, (uint64_t)(64u + 16u + 16u * (nfull + 1u)) * 8u);
            if (PERKEY)
                load8(opad, r + REC_OPAD);
            else
                load_uniform8(opad, a.rec + REC_OPAD);
            hmac_finish(h, tu >= 4u ? 0u : 1u, w, fin, opad);
            if (valid) {
                uint8_t *T = O + US * (nfull + 2u);
                st16(T, u32x4{bswap(h[0]), bswap(h[1]), bswap(h[2]), bswap(h[3])});
                st16(T + US, u32x4{bswap(h[4]), bswap(h[5]), bswap(h[6]), bswap(h[7])});
            }
        }
    }
#ifdef RNSTOK_SPLIT_PROBE
    if (lane == 0u) {
        const uint32_t r = aes ? 0u : 1u;
        atomicAdd(&g_split_probe[r], pr_wait);
        atomicAdd(&g_split_probe[2 + r], pr_n);
        atomicAdd(&g_split_probe[4 + r], clock64() - pr_t0);
        atomicAdd(&g_split_probe[6 + r], 1ull);
    }
#endif
    clk.finish(a.clk);
}

// ---------------------------------------------------- encrypt, long tokens --
//
// Few, long tokens (e.g. 16 KiB Resource segments sharded over 8 GPUs leave
// 128 tokens per CU): one packet per lane no longer fills the machine, and
// each lane's AES chain (latency-bound on LDS) and SHA chain (VALU) would run
// back to back.  Here a workgroup of 2*G waves serves G groups of 64 tokens:
// wave g (< G) runs the CBC chains of group g and drops each quad of
// ciphertext into an LDS ring; wave G+g hashes the previous quad of the same
// group.  One __syncthreads() per quad step keeps producer and consumer one
// step apart (double-buffered ring after the 128 KiB table image).
constexpr uint32_t RING_BASE = LDS_ENC_BYTES;                 // 0x20000
constexpr uint32_t RING_BYTES = 2u * 2u * 64u * 64u;                           // G <= 2 groups x 2 slots
constexpr uint32_t STEP_WORD = RING_BASE + RING_BYTES;                         // workgroup max of quad steps
constexpr uint32_t LDS_ENC_LONG_BYTES = STEP_WORD + 16u;
// (no static __shared__ here: the absolute LDS addresses assume the dynamic
// region starts at 0)

__device__ __forceinline__ void ring_put(uint32_t grp, uint32_t slot, uint32_t lane, const u32x4 c[4]) {
    typedef __attribute__((address_space(3))) u32x4 l128;
    l128 *r = (l128 *)(uintptr_t)(RING_BASE + ((grp * 2u + slot) * 64u + lane) * 64u);
    r[0] = c[0]; r[1] = c[1]; r[2] = c[2]; r[3] = c[3];
}
__device__ __forceinline__ void ring_get(uint32_t grp, uint32_t slot, uint32_t lane, u32x4 c[4]) {
    typedef __attribute__((address_space(3))) const u32x4 l128;
    l128 *r = (l128 *)(uintptr_t)(RING_BASE + ((grp * 2u + slot) * 64u + lane) * 64u);
    c[0] = r[0]; c[1] = r[1]; c[2] = r[2]; c[3] = r[3];
}

template <int NR, bool PERKEY>
__global__ __launch_bounds__(256) void k_encrypt_long(EncArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t tab_u32[];
    typedef __attribute__((address_space(3))) uint32_t lds_word;
    lds_word *max_steps = (lds_word *)(uintptr_t)STEP_WORD;
    LaunchClock clk;
    clk.start(a.clk);
    fill_tables<false>(tab_u32, a.sbox, a.sbox + 256);
    const Lanes LN(threadIdx.x & 31u);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint32_t G = blockDim.x >> 7;
    const bool aes = wave < G;
    const uint32_t grp = aes ? wave : wave - G;
    const Layout in{a.pt_off, a.pt_stride, a.pt_len, a.uni_len};
    Keys<NR, PERKEY> K;
    if (!PERKEY && aes) K.load(a.rec, REC_ENC);

    for (uint32_t base = blockIdx.x * G * 64u; base < a.n; base += gridDim.x * G * 64u) {
        const uint32_t i = base + grp * 64u + lane;
        const bool valid = i < a.n;
        const uint32_t p = valid ? (a.order ? a.order[i] : i) : 0u;
        const uint32_t L = valid ? in.l(p) : 0u;
        const uint32_t nfull = L >> 4, nq = nfull >> 2, tb = (nfull & 3u) + 1u;
        const uint32_t steps = valid ? nq + 1u : 0u;          // full quads + the tail quad
        if (threadIdx.x == 0) *max_steps = 0;
        __syncthreads();
        __hip_atomic_fetch_max(max_steps, steps, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __syncthreads();
        const uint32_t Q = *max_steps;
        __syncthreads();          // everyone has read Q before the word is reset next iteration
        const uint8_t *P = a.pt + (valid ? in.o(p) : 0);
        uint8_t *O = a.tok + (valid ? (a.tok_off ? a.tok_off[p] : (uint64_t)p * a.tok_stride) : 0);
        const uint32_t *rec = PERKEY && valid ? a.rec + (uint64_t)a.key_idx[p] * REC_WORDS : a.rec;
        const u32x4 iv = valid ? ld16(a.iv + 16ull * p) : u32x4{0u, 0u, 0u, 0u};
        if (aes) {
            if (PERKEY && valid) K.load(rec, REC_ENC);
            Sha256 dummy;
            u32x4 prev = iv, x[4], c[4], xn[4];
            if (valid) st16(O, iv);
            if (nq > 0) { xn[0] = ld16(P); xn[1] = ld16(P + 16); xn[2] = ld16(P + 32); xn[3] = ld16(P + 48); }
            for (uint32_t k = 0; k < Q; ++k) {
                if (k < steps) {
                    const uint8_t *Pk = P + 64ull * k;
                    if (k < nq) {
                        // the next quad's plaintext is requested before this quad's rounds (HBM latency hidden)
                        x[0] = xn[0]; x[1] = xn[1]; x[2] = xn[2]; x[3] = xn[3];
                        if (k + 1 < nq) {
                            xn[0] = ld16(Pk + 64); xn[1] = ld16(Pk + 80); xn[2] = ld16(Pk + 96); xn[3] = ld16(Pk + 112);
                        }
                    } else {
                        const u32x4 z = {0u, 0u, 0u, 0u};
                        const uint32_t r = L & 15u;
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            x[j] = (uint32_t)j + 1u < tb ? ld16(Pk + 16 * j)
                                                         : ((uint32_t)j + 1u == tb ? pad_block(Pk + 16 * j, r) : z);
                    }
                    enc_quad<NR, false>(c, x, prev, K.rk, LN, dummy);
                    uint8_t *Ck = O + 16 + 64ull * k;
                    const uint32_t nst = k < nq ? 4u : tb;
                    st16(Ck, c[0]);
                    if (nst > 1) st16(Ck + 16, c[1]);
                    if (nst > 2) st16(Ck + 32, c[2]);
                    if (nst > 3) st16(Ck + 48, c[3]);
                    ring_put(grp, k & 1u, lane, c);
                    prev = c[3];
                }
                __syncthreads();     // quad k visible to the SHA wave; SHA done with slot (k-1)&1
            }
            __syncthreads();         // matches the consumer's final step
        } else {
            uint32_t h[8], opad[8];
            if (PERKEY) {
                if (valid) { load8(h, rec + REC_IPAD); load8(opad, rec + REC_OPAD); }
            } else {
                load_uniform8(h, a.rec + REC_IPAD);
                load_uniform8(opad, a.rec + REC_OPAD);
            }
            u32x4 prev = iv, c[4];
            const uint64_t bits = (uint64_t)(64u + 16u + 16u * (nfull + 1u)) * 8u;
            __syncthreads();         // step 0: nothing to hash yet
            for (uint32_t k = 1; k <= Q; ++k) {
                if (k <= steps) {
                    ring_get(grp, (k - 1) & 1u, lane, c);
                    if (k - 1 < nq) {
                        uint32_t w[16];
                        sha_units(w, prev, c[0], c[1], c[2]);
                        sha256_compress(h, w);
                        prev = c[3];
                    } else {
                        // tail quad: units prev, c[0..tb-1] (+ final padding), then the outer hash
                        const uint32_t tu = tb + 1;
                        if (tu >= 4) {
                            uint32_t w[16];
                            sha_units(w, prev, c[0], c[1], c[2]);
                            sha256_compress(h, w);
                            sha_final_units(h, tu - 4, c[3], c[3], c[3], bits);
                        } else {
                            sha_final_units(h, tu, prev, c[0], c[1], bits);
                        }
                        uint32_t tag[8];
                        hmac_outer(tag, h, opad);
                        uint8_t *T = O + 16 + 16ull * (nfull + 1u);
                        st16(T, u32x4{bswap(tag[0]), bswap(tag[1]), bswap(tag[2]), bswap(tag[3])});
                        st16(T + 16, u32x4{bswap(tag[4]), bswap(tag[5]), bswap(tag[6]), bswap(tag[7])});
                    }
                }
                __syncthreads();
            }
        }
    }
    clk.finish(a.clk);
}

// ------------------------------------ encrypt, long tokens, 4 lanes/token --
//
// c4 sharded over 8 GPUs leaves 128 tokens of 16 KiB per CU, and a token's
// CBC chain (1025 blocks x NR rounds, each round waiting on its table
// lookups) is the critical path.  Here a quad of lanes carries one chain:
// lane j owns column j of the state and looks up the four bytes of ITS column
// word (T0[s_j.b0] feeds column j, T1[s_j.b1] column j-1, T2[s_j.b2] column
// j-2, T3[s_j.b3] column j-3), then gathers the other three terms of its
// column from the quad with DPP quad permutes: 3 addresses + 4 lookups + 4
// XORs per lane and round instead of 16 + 16 + 8, so a round costs one LDS
// round trip plus a few VALU cycles.  Waves 0-7 run the chains of 128 tokens
// (16 per wave) and drop each quad of ciphertext into a two-slot LDS ring;
// waves 8-9 hash the previous quad of the same tokens, one token per lane,
// one barrier per quad step.  Single key, uniform lengths.
// Hashing waves: 4 (one per SIMD, 32 tokens each) measured 8 % slower than 2
// on the c4 shard (profiles/r03g_long4_ab.txt).
constexpr uint32_t L4_TOK = 128, L4_AES_WAVES = 8, L4_HASH_WAVES = 2;
constexpr uint32_t L4_THREADS = 64u * (L4_AES_WAVES + L4_HASH_WAVES), L4_HASH_TOK = L4_TOK / L4_HASH_WAVES;
static_assert(L4_HASH_TOK <= 64u && L4_TOK % L4_HASH_WAVES == 0u, "one token per hashing lane");

// Ring layout: token t's quad (4 blocks x 16 B) at t*64 B.  The AES lanes'
// 4-B stores (lanes of 8 consecutive tokens x 4 columns) meet 4-way and the
// hashing lanes' 16-B reads (one token per lane) 4-way bank conflicts (7 % of
// the kernel's LDS cycles, profiles/r02e_c4s8_pmc_summary.txt).  A swizzle
// that makes both conflict-free (block i in 16-B unit i ^ (((t >> 1) ^ (t >>
// 2)) & 3)) measured 1.2 % slower on the c4 shard (1.001 vs 0.989 ms,
// profiles/r03g_long4_ab.txt): the LDS pipe is not what bounds this kernel.
constexpr uint32_t L4_RING = LDS_ENC_BYTES;                              // after the table image
// The ring holds 2 quads per token: AES waves fill one per barrier while the
// hashing waves consume the other.  Two quads per phase (half the barriers, a
// 160 KiB image) measured the same as one (c4 shard 0.999 vs 0.997 ms): the
// fused kernel's excess over its AES side alone (0.91 ms; hashing side alone
// 0.73) is SIMD contention, not barrier jitter.
constexpr uint32_t L4_SLOTS = 2u;
// Waves none of whose lanes holds a token of the batch skip the rounds and
// only meet the barriers.  In a launch of a few tokens (one Token call) their
// chains on garbage took issue slots from the live AES and hashing chains
// that share their SIMDs.
#ifndef RNSTOK_L4_SKIP_IDLE
#define RNSTOK_L4_SKIP_IDLE 1
#endif
#ifndef RNSTOK_L4_HASH_FIRST
#define RNSTOK_L4_HASH_FIRST 1
#endif
constexpr uint32_t LDS_ENC_LONG4_BYTES = L4_RING + L4_SLOTS * L4_TOK * 64u;   // + 2 slots x 128 tokens x 64 B

// DPP quad_perm: lane j of each group of four reads lane (j + K) & 3.
template <int K>
__device__ __forceinline__ uint32_t quad_rot(uint32_t v) {
    constexpr int ctrl = K == 1 ? 0x39 : (K == 2 ? 0x4E : 0x93);
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, ctrl, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t ld32u(const uint8_t *p) {
    uint32_t v;
    __builtin_memcpy(&v, p, 4);
    return v;
}
__device__ __forceinline__ void st32u(uint8_t *p, uint32_t v) { __builtin_memcpy(p, &v, 4); }

// Column `col` (bytes 4col..4col+3) of the PKCS7 pad block with r payload bytes at p.
__device__ __forceinline__ uint32_t pad_col(const uint8_t *p, uint32_t r, uint32_t col) {
    uint32_t w = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t i = 4u * col + (uint32_t)k;
        w |= (i < r ? (uint32_t)p[i] : 16u - r) << (8 * k);
    }
    return w;
}

// One block of the chain on a quad of lanes: s = this lane's column of
// plaintext ^ previous ciphertext, rk = this lane's round-key column;
// returns this lane's ciphertext column.
template <int NR>
__device__ __forceinline__ uint32_t enc_block4(uint32_t s, const uint32_t *rk, const Lanes &L) {
    s ^= rk[0];
#pragma unroll
    for (int r = 1; r < NR; ++r) {
        const uint32_t u0 = lds(taddr<0, 0>(s, L), 0), u1 = lds(taddr<1, 0>(s, L), 128);
        const uint32_t u2 = lds(taddr<2, 1>(s, L), 0), u3 = lds(taddr<3, 1>(s, L), 128);
        // three independent DPP moves, then two xor3: the chain is latency-
        // bound, and this is a shorter dependent path than the three
        // v_xor_b32_dpp in a row the compiler folds the plain XORs into
        // (c4 shard encrypt 1.044 -> 0.992 ms, A/B)
        // (Two of the moves carrying an XOR, v_xor_b32 with a DPP source,
        // and one xor3 after them: 12 instructions per round instead of 13
        // but 3.8 % slower on the c4 shard, profiles/r03g_long4_ab.txt.)
        uint32_t x1 = quad_rot<1>(u1), x2 = quad_rot<2>(u2), x3 = quad_rot<3>(u3);
        asm volatile("" : "+v"(x1), "+v"(x2), "+v"(x3));
        s = xor3(xor3(x1, x2, x3), u0, rk[r]);
    }
    // final round: byte k of column j is S[s_{j+k}.b_k] (tlast_enc, split the same way)
    const uint32_t v0 = lds(taddr<0, 1>(s, L), 0) & 0x000000ffu, v1 = lds(taddr<1, 1>(s, L), 128) & 0x0000ff00u;
    const uint32_t v2 = lds(taddr<2, 0>(s, L), 0) & 0x00ff0000u, v3 = lds(taddr<3, 0>(s, L), 128) & 0xff000000u;
    uint32_t x1 = quad_rot<1>(v1), x2 = quad_rot<2>(v2), x3 = quad_rot<3>(v3);
    asm volatile("" : "+v"(x1), "+v"(x2), "+v"(x3));
    return xor3(xor3(x1, x2, x3), v0, rk[NR]);
}

template <int NR>
__global__ __launch_bounds__(L4_THREADS) void k_encrypt_long4(EncArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t tab_u32[];
    typedef __attribute__((address_space(3))) uint32_t lds_w;
    typedef __attribute__((address_space(3))) const u32x4 lds_q;
    LaunchClock clk;
    clk.start(a.clk);
    const Lanes LN(threadIdx.x & 31u);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    // RNSTOK_L4_HASH_FIRST: in a launch of at most 64 tokens the hashing
    // waves are waves 0-1 and the first tokens' AES wave is wave 2, so its
    // AES and hashing chains run on different SIMDs (else waves 0 and 8 shared
    // SIMD 0): one 383-B token -2 %.  Full workgroups keep the AES waves
    // first: hashing first there cost the c4 rank share's encrypt 2.24 ->
    // 3.39 M cycles (profiles/r06_latency_kernels/c4_share_hash_first.txt).
    const bool hf = RNSTOK_L4_HASH_FIRST && a.n <= L4_HASH_TOK;                 // launch-uniform
    const uint32_t hw = hf ? (wave < L4_HASH_WAVES ? L4_AES_WAVES + wave : wave - L4_HASH_WAVES) : wave;
    const bool aes = hw < L4_AES_WAVES;
    const uint32_t col = threadIdx.x & 3u;
    const bool hash_lane = aes || lane < L4_HASH_TOK;
    const uint32_t slot = aes ? (64u * hw + lane) >> 2 : (hw - L4_AES_WAVES) * L4_HASH_TOK + (hash_lane ? lane : 0u);
    const uint32_t L = a.uni_len, nfull = L >> 4, nq = nfull >> 2, tb = (nfull & 3u) + 1u, rem = L & 15u;
    uint32_t rk[NR + 1];
#pragma unroll
    for (int r = 0; r <= NR; ++r) rk[r] = aes ? a.rec[REC_ENC + 4 * r + col] : 0u;

    for (uint32_t base = blockIdx.x * L4_TOK; base < a.n; base += gridDim.x * L4_TOK) {
        const uint32_t t = base + slot;
        const bool valid = t < a.n && hash_lane;
        const uint32_t p = valid ? (a.order ? a.order[t] : t) : 0u;
        const uint8_t *P = a.pt + (valid ? in_off(a.pt_off, a.pt_stride, p) : 0);
        uint8_t *O = a.tok + (valid ? in_off(a.tok_off, a.tok_stride, p) : 0);
        const bool live = !RNSTOK_L4_SKIP_IDLE || __ballot(valid) != 0ull;     // wave-uniform
        // this lane's column of the plaintext blocks of quad k (the tail quad: tb blocks, the last padded)
        auto load_quad = [&](uint32_t k, uint32_t x[4]) {
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const uint8_t *B = P + 16ull * (4u * k + (uint32_t)b);
                x[b] = !valid ? 0u
                              : ((k < nq || (uint32_t)b + 1u < tb) ? ld32u(B + 4u * col)
                                                                    : ((uint32_t)b + 1u == tb ? pad_col(B, rem, col) : 0u));
            }
        };
        // The batch's IV (each AES lane's column, each hashing lane's whole
        // unit) and first quad are requested before the first batch's table
        // fill: for a Token call they sit in the pinned staging buffer, and
        // the fill hides that PCIe round trip.
        uint32_t prev = 0u, xn[4] = {0u, 0u, 0u, 0u};
        u32x4 hiv = {0u, 0u, 0u, 0u};
        if (aes) {
            prev = valid ? ld32u(a.iv + 16ull * p + 4u * col) : 0u;
            load_quad(0u, xn);
        } else if (valid) {
            hiv = ld16(a.iv + 16ull * p);
        }
        if (base == blockIdx.x * L4_TOK) fill_tables<false>(tab_u32, a.sbox, a.sbox + 256);   // (workgroup-uniform)
        if (aes) {
            if (valid) st32u(O + 4u * col, prev);
            for (uint32_t k = 0; k <= nq; ++k) {
                const uint32_t x[4] = {xn[0], xn[1], xn[2], xn[3]};
                if (k < nq) load_quad(k + 1u, xn);        // the next quad is requested before this quad's rounds
                uint32_t cq[4] = {0u, 0u, 0u, 0u};
                if (live) {
#pragma unroll
                    for (int b = 0; b < 4; ++b) {
#ifndef RNSTOK_L4_PROBE_SHA_ONLY        // timing probe: no AES (wrong tokens)
                        cq[b] = enc_block4<NR>(x[b] ^ prev, rk, LN);
#else
                        cq[b] = x[b] ^ prev;
#endif
                        prev = cq[b];
                    }
                }
                const uint32_t nst = k < nq ? 4u : tb;
                uint8_t *Ck = O + 16 + 64ull * k + 4u * col;
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    if (valid && (uint32_t)b < nst) st32u(Ck + 16 * b, cq[b]);
                lds_w *ring = (lds_w *)(uintptr_t)(L4_RING + ((k % L4_SLOTS) * L4_TOK + slot) * 64u + 4u * col);
#pragma unroll
                for (int b = 0; b < 4; ++b) ring[4u * (uint32_t)b] = cq[b];
                // the quad becomes visible to the hashing waves, which are
                // done with the previous one's slot
                __syncthreads();
            }
            __syncthreads();         // matches the hashing waves' last phase
        } else {
            uint32_t h[8], opad[8];
            load_uniform8(h, a.rec + REC_IPAD);
            load_uniform8(opad, a.rec + REC_OPAD);
            u32x4 prev = hiv;
            const uint64_t bits = (uint64_t)(64u + 16u + 16u * (nfull + 1u)) * 8u;
            __syncthreads();         // step 0: nothing to hash yet
            for (uint32_t q = 0; q <= nq; ++q) {
                lds_q *r = (lds_q *)(uintptr_t)(L4_RING + ((q % L4_SLOTS) * L4_TOK + slot) * 64u);
                const u32x4 c0 = r[0], c1 = r[1], c2 = r[2], c3 = r[3];
                if (q < nq) {
#ifndef RNSTOK_L4_PROBE_AES_ONLY        // timing probe: no HMAC (wrong tags)
                    if (live) {
                        uint32_t w[16];
                        sha_units(w, prev, c0, c1, c2);
                        sha256_compress(h, w);
                    }
#endif
                    prev = c3;
                } else if (valid) {
                    // tail quad: units prev, c0..c_{tb-1} (+ final padding), then the outer hash
                    const uint32_t tu = tb + 1u;
                    if (tu >= 4u) {
                        uint32_t w[16];
                        sha_units(w, prev, c0, c1, c2);
                        sha256_compress(h, w);
                        sha_final_units(h, tu - 4u, c3, c3, c3, bits);
                    } else {
                        sha_final_units(h, tu, prev, c0, c1, bits);
                    }
                    uint32_t tag[8];
                    hmac_outer(tag, h, opad);
                    uint8_t *T = O + 16 + 16ull * (nfull + 1u);
                    st16(T, u32x4{bswap(tag[0]), bswap(tag[1]), bswap(tag[2]), bswap(tag[3])});
                    st16(T + 16, u32x4{bswap(tag[4]), bswap(tag[5]), bswap(tag[6]), bswap(tag[7])});
                }
                __syncthreads();
            }
        }
    }
    clk.finish(a.clk);
}

// --------------------------------------------------------------- decrypt --


// WG: the workgroup size the kernel is compiled for (its VGPR budget).  One
// key: 768 threads (168 VGPRs) for batches of several passes, 1024 (128
// VGPRs, 4 waves/SIMD) when one pass covers the batch (e.g. 16 KiB Resource
// tokens, one per lane: 512 x 2 passes at 768 was 9 % slower).
template <int NR, bool PERKEY, int WG = PERKEY ? WG_PERKEY_DEC : WG_DEC, bool ILV = false>
__global__ RT_OCC __launch_bounds__(WG) void k_decrypt(DecArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t tab_u32[];
    LaunchClock clk;
    clk.start(a.clk);
    fill_tables<true>(tab_u32, a.sbox, a.sbox + 256);
    const Lanes LN(threadIdx.x & 31u);

    Keys<NR, PERKEY> K;
    uint32_t ipad[8], opad[8];
    if (!PERKEY) K.load(a.rec, REC_DEC);
    const Layout in{a.tok_off, a.tok_stride, a.tok_len, a.uni_len};

    RT_PACKET_LOOP(a, i) {
        const uint32_t p = a.order ? a.order[i] : i;
        const uint32_t *r = PERKEY ? a.rec + (uint64_t)a.key_idx[p] * REC_WORDS : a.rec;
        if (PERKEY) {
            K.load(r, REC_DEC);
            load8(ipad, r + REC_IPAD);
        } else {
            load_uniform8(ipad, a.rec + REC_IPAD);
        }
        // opad: loaded where it is used, after the quad loop
        const uint32_t T = in.l(p);
        const uint64_t US = ILV ? 16ull * a.n : 16ull;       // see k_encrypt
        const uint8_t *Kt = ILV ? a.tok + 16ull * p : a.tok + in.o(p);
        uint8_t *O = ILV ? a.pt + 16ull * p : a.pt + (a.pt_off ? a.pt_off[p] : (uint64_t)p * a.pt_stride);
        int32_t st;
        uint32_t outlen = 0;

        // (the interleaved layout takes well-formed uniform tokens only: rt_decrypt_interleaved)
        if (!ILV && (T < 64u || ((T - 48u) & 15u))) {
            // Malformed length (rare): decide TOO_SHORT / BAD_HMAC / BAD_CT_LEN
            // exactly as Token.decrypt would, without touching the AES path.
            if (T <= 32u) {
                st = 1;
            } else {
                uint32_t h[8], tag[8];
                for (int i = 0; i < 8; ++i) h[i] = ipad[i];
                if (PERKEY)
                    load8(opad, r + REC_OPAD);
                else
                    load_uniform8(opad, a.rec + REC_OPAD);
                sha_bytes_after_ipad(h, Kt, T - 32u);
                hmac_outer(tag, h, opad);
                uint32_t diff = 0;
                for (int i = 0; i < 32; ++i) diff |= (uint32_t)Kt[T - 32u + i] ^ ((tag[i >> 2] >> (24 - 8 * (i & 3))) & 0xffu);
                st = diff ? 2 : 3;
            }
            if (T > 48u)   // caller's region holds T-48 bytes: zero it
                for (uint32_t i = 0; i < T - 48u; ++i) O[i] = 0;
        } else {
            const uint32_t nb = (T - 48u) >> 4, nq = (nb - 1u) >> 2, tb = ((nb - 1u) & 3u) + 1u;
            uint32_t h[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) h[i] = ipad[i];
            // One dec_quad instance serves every quad, the tail quad (tb
            // blocks) included; its SHA slot hashes the same quad's units
            // (dropped for a tail of tb < 3, whose units are not a full
            // block).  hmac_finish runs the final block and the outer hash
            // through one sha256_compress.
            const u32x4 z = {0u, 0u, 0u, 0u};
            u32x4 prev = ld16(Kt);
            // (RNSTOK_DEC_TAG_EARLY: the tag's two units loaded before the quad
            // loop, so the compare after it does not wait on them)
            constexpr bool TAG_EARLY = RNSTOK_DEC_TAG_EARLY && !PERKEY && WG <= 768;
            u32x4 tag0, tag1;
            if (TAG_EARLY) {
                tag0 = ld16(Kt + US * ((T >> 4) - 2u));
                tag1 = ld16(Kt + US * ((T >> 4) - 1u));
            }
            const uint8_t *C = Kt + US;
            uint8_t *D = O;
            Sha256 S;
            u32x4 c[4], pp[4];
            // packed rows: an even quad loads the next quad's 64 B with its
            // own, so the 128-B line the two share is read while it is in
            // L2 (one quad apart, an XCD's waves have streamed more than its
            // L2 through and the line is fetched again: 2.7x read traffic)
            constexpr bool PAIR = RNSTOK_DEC_PAIR && !ILV && !PERKEY && WG <= 768;   // (1024: 11 -> 38 VGPRs spilled)
            u32x4 nx[4];
#pragma nounroll
            for (uint32_t q = 0; q <= nq; ++q) {
                const uint32_t nbk = q < nq ? 4u : tb;
                if (PAIR && (q & 1u)) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) c[k] = nx[k];
                } else {
                    c[0] = ld16(C);
                    c[1] = nbk > 1u ? ld16(C + US) : z;
                    c[2] = nbk > 2u ? ld16(C + 2 * US) : z;
                    c[3] = nbk > 3u ? ld16(C + 3 * US) : z;
                    if (PAIR && q < nq) {
                        const uint32_t nb1 = q + 1u < nq ? 4u : tb;
                        nx[0] = ld16(C + 4 * US);
                        nx[1] = nb1 > 1u ? ld16(C + 5 * US) : z;
                        nx[2] = nb1 > 2u ? ld16(C + 6 * US) : z;
                        nx[3] = nb1 > 3u ? ld16(C + 7 * US) : z;
                    }
                }
                S.start(h);
                sha_units(S.w, prev, c[0], c[1], c[2]);
                dec_quad<NR, true>(pp, c, prev, K.rk, LN, S);
#pragma unroll
                for (int k = 0; k < 8; ++k) asm volatile("" ::"v"(S.v[k]));   // see k_encrypt
                const bool keep = nbk >= 3u;
#pragma unroll
                for (int k = 0; k < 8; ++k) h[k] += keep ? S.v[k] : 0u;
                st16(D, pp[0]);
                if (nbk > 1u) st16(D + US, pp[1]);
                if (nbk > 2u) st16(D + 2 * US, pp[2]);
                if (nbk > 3u) st16(D + 3 * US, pp[3]);
                prev = c[3];
                C += 4 * US; D += 4 * US;
            }
            // the tail quad: pb = the block before it (re-read rather than
            // kept live through the loop), c[0..tb-1] its ciphertext,
            // pp[0..tb-1] its plaintext
            const u32x4 pb = ld16(Kt + 4ull * US * nq);
            u32x4 r0, r1;
            if (TAG_EARLY) {
                r0 = tag0;
                r1 = tag1;
            } else {
                r0 = ld16(Kt + US * ((T >> 4) - 2u));
                r1 = ld16(Kt + US * ((T >> 4) - 1u));
            }
            const u32x4 last = tb == 1u ? pp[0] : (tb == 2u ? pp[1] : (tb == 3u ? pp[2] : pp[3]));
            const bool full = tb >= 3u;
            const uint32_t tu = tb + 1u;
            uint32_t u[16], fin[16];
            sha_units(u, full ? c[3] : pb, c[0], c[1], z);
            sha_final_block(fin, u, full ? tu - 4u : tu, (uint64_t)(64u + 16u + 16u * nb) * 8u);
            if (PERKEY)
                load8(opad, r + REC_OPAD);
            else
                load_uniform8(opad, a.rec + REC_OPAD);
            hmac_finish(h, 1u, fin, fin, opad);
            const uint32_t diff = (r0.x ^ bswap(h[0])) | (r0.y ^ bswap(h[1])) | (r0.z ^ bswap(h[2])) |
                                  (r0.w ^ bswap(h[3])) | (r1.x ^ bswap(h[4])) | (r1.y ^ bswap(h[5])) |
                                  (r1.z ^ bswap(h[6])) | (r1.w ^ bswap(h[7]));
            const uint32_t padn = last.w >> 24;     // PKCS7.unpad: n = data[-1]
            st = diff ? 2 : (padn > 16u ? 4 : 0);
            if (st == 0) {
                outlen = 16u * nb - padn;
            } else {
                if (st == 4) outlen = padn;   // authenticated pad byte, for the error message
                for (uint32_t i = 0; i < nb; ++i) st16(O + US * i, z);
            }
        }
        a.status[p] = st;
        a.out_len[p] = outlen;
    }
    clk.finish(a.clk);
}

// ---------------------------------------------------- decrypt, long tokens --
//
// Few, long tokens, one key, uniform length T (48 + 16*nb, nb >= 61), e.g.
// the 16 KiB Resource segments of c4 sharded 8 ways (128 per CU).  CBC
// decryption is block-parallel; only the HMAC is a serial chain, with the
// message schedule moved off it.  A token's 257 compressions are one serial
// chain in one lane; one wave issues at most one VALU instruction per ~4 cycles, so
// the chain's time is its instruction count.  W[16..63] depends only on the
// message, not on the state, so here producer waves compute W[t] + K[t] for
// every block and hand it to the chain (consumer) waves through an LDS ring:
// the chain issues 14 instructions per round instead of ~21.5 (rounds plus
// schedule), i.e. ~35 % fewer.
//
//   waves 0-1  consumers: the HMAC chains of 64 tokens each (one per lane)
//   waves 2-3  producers: the schedules of the same 64 tokens, one block ahead
//   waves 4-   block-parallel CBC decryption of the batch's quads, taken 64
//              at a time from an LDS counter (SIMD balance)
//
// Producer p and consumer p pair through two LDS counters (steps written,
// steps consumed) with a two-slot ring; no workgroup barrier inside the
// chain, so the AES waves never wait on it.  The LDS image makes room for the
// 64 KiB ring: T0/T1 only (Td2 = rotl16(Td0), Td3 = rotl16(Td1), one
// v_alignbit per column on the XOR of the two lookups) and a 16-replica InvS.
#ifndef RNSTOK_DL2_AES_WAVES
#define RNSTOK_DL2_AES_WAVES 12
#endif
constexpr uint32_t DL2_TOK = 128, DL2_AES_WAVES = RNSTOK_DL2_AES_WAVES, DL2_THREADS = 64u * (4u + DL2_AES_WAVES);
constexpr uint32_t DL2_INVS = 0x10000;                       // 256 rows x 64 B: InvS[x]*0x01010101 x16
constexpr uint32_t DL2_RING = 0x14000;                       // 2 slots x 16 quads x 128 tokens x 16 B
constexpr uint32_t DL2_SLOT = 16u * DL2_TOK * 16u;           // 32 KiB
constexpr uint32_t DL2_FLAGS = DL2_RING + 2u * DL2_SLOT;     // ready[2], done[2] (u32)
constexpr uint32_t DL2_PADN = DL2_FLAGS + 64u;                // per token of the batch: its last plaintext byte
constexpr uint32_t LDS_DL2_BYTES = DL2_PADN + 4u * DL2_TOK;
// The producers also schedule the final padded block, so the chain runs it
// from the ring like the others (its own schedule inline took a third more
// instructions per round).
#ifndef RNSTOK_DL2_FINAL
#define RNSTOK_DL2_FINAL 1
#endif
constexpr bool DL2_FINAL = RNSTOK_DL2_FINAL;
#ifndef RNSTOK_DL2_SKIP_IDLE
#define RNSTOK_DL2_SKIP_IDLE 1
#endif
constexpr bool DL2_SKIP_IDLE = RNSTOK_DL2_SKIP_IDLE;

__device__ void fill_tables_dl2(uint32_t *tab, const uint8_t *inv) {
    const uint32_t lane = threadIdx.x & 31u;
    for (uint32_t u = threadIdx.x; u < 512u; u += blockDim.x) {        // Td0, Td1 (region 0 only)
        const uint32_t x = u & 255u, t = u >> 8;
        const uint32_t v = rotl(td0(inv, x), 8 * (int)t);
        uint32_t *row = tab + (x << 6) + (t << 5);
#pragma unroll 8
        for (uint32_t j = 0; j < 32u; ++j) row[(j + lane) & 31u] = v;
    }
    for (uint32_t x = threadIdx.x; x < 256u; x += blockDim.x) {
        const uint32_t v = (uint32_t)inv[x] * 0x01010101u;
        uint32_t *row = tab + (DL2_INVS >> 2) + (x << 4);
#pragma unroll
        for (uint32_t j = 0; j < 16u; ++j) row[(j + lane) & 15u] = v;
    }
    if (threadIdx.x < 16u) tab[(DL2_FLAGS >> 2) + threadIdx.x] = 0u;
    __syncthreads();
}

// InvS[byte K of s] from 64-B rows of 16 replicas (lane l reads replica l & 15)
template <int K>
__device__ __forceinline__ uint32_t invs16(uint32_t s, uint32_t lane_off) {
    const uint32_t t = K == 0 ? (s << 6) : (s >> (8 * K - 6));
    return lds(and_or(t, 0x3fc0u, lane_off), 0);
}

// Equivalent inverse cipher on 4 independent blocks with Td0/Td1 only:
// Td2[x] ^ Td3[y] = rotl16(Td0[x] ^ Td1[y]).
template <int NR>
__device__ __forceinline__ void dec_quad_t01(u32x4 p[4], const u32x4 c[4], u32x4 chain, const uint32_t *dk,
                                             const Lanes &L, uint32_t inv_off) {
    uint32_t s[4][4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        s[b][0] = c[b].x ^ dk[0]; s[b][1] = c[b].y ^ dk[1]; s[b][2] = c[b].z ^ dk[2]; s[b][3] = c[b].w ^ dk[3];
    }
#pragma unroll
    for (int r = 1; r < NR; ++r) {
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            uint32_t v[16];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                v[4 * j + 0] = lds(taddr<0, 0>(s[b][j], L), 0);
                v[4 * j + 1] = lds(taddr<1, 0>(s[b][(j + 3) & 3], L), 128);
                v[4 * j + 2] = lds(taddr<2, 0>(s[b][(j + 2) & 3], L), 0);
                v[4 * j + 3] = lds(taddr<3, 0>(s[b][(j + 1) & 3], L), 128);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t hi = v[4 * j + 2] ^ v[4 * j + 3];
                s[b][j] = xor3(v[4 * j], v[4 * j + 1], rotr(hi, 16)) ^ dk[4 * r + j];
            }
        }
    }
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const uint32_t *t = s[b];
        u32x4 o;
        o.x = bfi(0x0000ffffu, bfi(0x000000ffu, invs16<0>(t[0], inv_off), invs16<1>(t[3], inv_off)),
                  bfi(0x00ff0000u, invs16<2>(t[2], inv_off), invs16<3>(t[1], inv_off))) ^ dk[4 * NR + 0];
        o.y = bfi(0x0000ffffu, bfi(0x000000ffu, invs16<0>(t[1], inv_off), invs16<1>(t[0], inv_off)),
                  bfi(0x00ff0000u, invs16<2>(t[3], inv_off), invs16<3>(t[2], inv_off))) ^ dk[4 * NR + 1];
        o.z = bfi(0x0000ffffu, bfi(0x000000ffu, invs16<0>(t[2], inv_off), invs16<1>(t[1], inv_off)),
                  bfi(0x00ff0000u, invs16<2>(t[0], inv_off), invs16<3>(t[3], inv_off))) ^ dk[4 * NR + 2];
        o.w = bfi(0x0000ffffu, bfi(0x000000ffu, invs16<0>(t[3], inv_off), invs16<1>(t[2], inv_off)),
                  bfi(0x00ff0000u, invs16<2>(t[1], inv_off), invs16<3>(t[0], inv_off))) ^ dk[4 * NR + 3];
        p[b] = o ^ (b == 0 ? chain : c[b - 1]);
    }
}

typedef __attribute__((address_space(3))) uint32_t lds_word_t;
typedef __attribute__((address_space(3))) u32x4 lds_quad_t;

__device__ __forceinline__ void dl2_wait(uint32_t flag_addr, uint32_t v) {
    lds_word_t *f = (lds_word_t *)(uintptr_t)flag_addr;
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < v) __builtin_amdgcn_s_sleep(1);
}
__device__ __forceinline__ void dl2_signal(uint32_t flag_addr, uint32_t v) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");      // the wave's ring accesses are done
    if ((threadIdx.x & 63u) == 0u)
        __hip_atomic_store((lds_word_t *)(uintptr_t)flag_addr, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <int NR>
__global__ __launch_bounds__(DL2_THREADS) void k_decrypt_long2(DecArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint32_t tab_u32[];
    LaunchClock clk;
    clk.start(a.clk);
    fill_tables_dl2(tab_u32, a.sbox + 256);
    const Lanes LN(threadIdx.x & 31u);
    const uint32_t inv_off = DL2_INVS | (4u * (threadIdx.x & 15u));
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint32_t T = a.uni_len, nb = (T - 48u) >> 4, nquads = (nb + 3u) >> 2, tbl = nb - 4u * (nquads - 1u);
    const uint32_t M = T - 32u, full = M >> 6;                 // full = 0 for a 64-B token: no chain steps
#if defined(RNSTOK_DL2_PROBE_AES_ONLY)          // timing probes (wrong statuses): one side of the kernel only
    const bool consumer = false, producer = false;
    if (wave < 4u) {
        __syncthreads();
        __syncthreads();
        for (uint32_t base = blockIdx.x * DL2_TOK + gridDim.x * DL2_TOK; base < a.n; base += gridDim.x * DL2_TOK) {
            __syncthreads();
            __syncthreads();
        }
        return;
    }
#else
    const bool consumer = wave < 2u, producer = wave == 2u || wave == 3u;
#endif
    const uint32_t pair = wave & 1u;                            // consumer p <-> producer p: tokens 64p..64p+63
    const uint32_t ready_f = DL2_FLAGS + 4u * pair, done_f = DL2_FLAGS + 8u + 4u * pair;
    Keys<NR, false> K;
    if (!consumer && !producer) K.load(a.rec, REC_DEC);

    for (uint32_t base = blockIdx.x * DL2_TOK; base < a.n; base += gridDim.x * DL2_TOK) {
        const uint32_t ntok = a.n - base < DL2_TOK ? a.n - base : DL2_TOK;
        const uint32_t slot_tok = pair * 64u + lane;            // this lane's column of the ring
        uint32_t diff = 1;
        // DL2_SKIP_IDLE: a batch of at most 64 tokens leaves chain pair 1
        // without a token; it skips its chains, and only the AES waves on
        // SIMDs 1 and 3 take quads, so the live chain waves (0 on SIMD 0, 2 on
        // SIMD 2) share their SIMDs with nothing (one Token call)
        const bool idle = DL2_SKIP_IDLE && ((consumer || producer) ? pair * 64u >= ntok : (ntok <= 64u && !(wave & 1u)));
        if (idle) {
        } else if (producer) {
            // tokens past the batch hash a copy of its last token (results unused)
            const uint32_t t = base + (slot_tok < ntok ? slot_tok : ntok - 1u);
            const uint8_t *Kt = a.tok + in_off(a.tok_off, a.tok_stride, a.order ? a.order[t] : t);
            // the final padded block (the last fu units of iv || ct) too, with DL2_FINAL
            const uint32_t fu = (M - 64u * full) >> 4, nblk = full + (DL2_FINAL ? 1u : 0u);
            const u32x4 z = {0u, 0u, 0u, 0u};
            auto load_block = [&](uint32_t i, u32x4 &c0, u32x4 &c1, u32x4 &c2, u32x4 &c3) {
                const uint8_t *B = Kt + 64ull * i;
                const uint32_t nu = i < full ? 4u : fu;         // (the final block's units stop at the tag)
                c0 = nu > 0u ? ld16(B) : z; c1 = nu > 1u ? ld16(B + 16) : z;
                c2 = nu > 2u ? ld16(B + 32) : z; c3 = nu > 3u ? ld16(B + 48) : z;
            };
            u32x4 b0, b1, b2, b3;
            load_block(0u, b0, b1, b2, b3);
            for (uint32_t i = 0; i < nblk; ++i) {
                uint32_t w[16];
                sha_units(w, b0, b1, b2, b3);
                if (DL2_FINAL && i == full) {
                    uint32_t fin[16];
                    sha_final_block(fin, w, fu, (uint64_t)(64u + M) * 8u);
#pragma unroll
                    for (int k = 0; k < 16; ++k) w[k] = fin[k];
                }
                if (i + 1 < nblk) load_block(i + 1u, b0, b1, b2, b3);     // next block requested before this schedule
                if (i >= 2u) dl2_wait(done_f, i - 1u);           // the consumer is done with slot i & 1
                lds_quad_t *ring = (lds_quad_t *)(uintptr_t)(DL2_RING + (i & 1u) * DL2_SLOT) + slot_tok;
                constexpr uint32_t Kc[64] = {
                    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
                    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
                    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
                    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
                    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
                    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
                    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
                    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    uint32_t wk[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int t4 = 4 * q + j;
                        uint32_t wt;
                        if (t4 < 16) {
                            wt = w[t4];
                        } else {
                            const uint32_t w15 = w[(t4 + 1) & 15], w2 = w[(t4 + 14) & 15];
                            const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
                            const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
                            wt = w[t4 & 15] = (w[t4 & 15] + s0 + w[(t4 + 9) & 15]) + s1;
                        }
                        wk[j] = wt + Kc[t4];
                    }
                    ring[q * DL2_TOK] = u32x4{wk[0], wk[1], wk[2], wk[3]};
                }
                dl2_signal(ready_f, i + 1u);
            }
        } else if (consumer) {
            const uint32_t t = base + slot_tok;
            const bool valid = slot_tok < ntok;
            const uint8_t *Kt = a.tok + in_off(a.tok_off, a.tok_stride,
                                               a.order ? a.order[valid ? t : base] : (valid ? t : base));
            uint32_t h[8], opad[8];
            load_uniform8(h, a.rec + REC_IPAD);
            // the tag, requested before the chain (a Token call's token sits in
            // pinned host memory: one PCIe round trip less at the end)
            const u32x4 r0 = ld16(Kt + M), r1 = ld16(Kt + M + 16);
            for (uint32_t i = 0; i < full + (DL2_FINAL ? 1u : 0u); ++i) {
                dl2_wait(ready_f, i + 1u);
                const lds_quad_t *ring = (const lds_quad_t *)(uintptr_t)(DL2_RING + (i & 1u) * DL2_SLOT) + slot_tok;
                uint32_t v[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] = h[k];
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const u32x4 wk4 = ring[q * DL2_TOK];
                    const uint32_t wk[4] = {wk4.x, wk4.y, wk4.z, wk4.w};
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int r = 4 * q + j;
                        const uint32_t A = v[(0 - r) & 7], B = v[(1 - r) & 7], C = v[(2 - r) & 7], D = v[(3 - r) & 7];
                        const uint32_t E = v[(4 - r) & 7], F = v[(5 - r) & 7], G = v[(6 - r) & 7], H = v[(7 - r) & 7];
                        const uint32_t t1 = (H + wk[j]) + xor3(rotr(E, 6), rotr(E, 11), rotr(E, 25)) + bfi(E, F, G);
                        const uint32_t t2 = xor3(rotr(A, 2), rotr(A, 13), rotr(A, 22)) + maj3(A, B, C);
                        v[(3 - r) & 7] = D + t1;
                        v[(7 - r) & 7] = t1 + t2;
                    }
                }
                dl2_signal(done_f, i + 1u);
#pragma unroll
                for (int k = 0; k < 8; ++k) h[k] += v[k];
            }
            if (!DL2_FINAL) {
                const uint32_t fu = (M - 64u * full) >> 4;
                const u32x4 z = {0u, 0u, 0u, 0u};
                const uint8_t *R = Kt + 64ull * full;
                sha_final_units(h, fu, fu > 0 ? ld16(R) : z, fu > 1 ? ld16(R + 16) : z, fu > 2 ? ld16(R + 32) : z,
                                (uint64_t)(64u + M) * 8u);
            }
            load_uniform8(opad, a.rec + REC_OPAD);
            uint32_t tag[8];
            hmac_outer(tag, h, opad);
            diff = (r0.x ^ bswap(tag[0])) | (r0.y ^ bswap(tag[1])) | (r0.z ^ bswap(tag[2])) |
                   (r0.w ^ bswap(tag[3])) | (r1.x ^ bswap(tag[4])) | (r1.y ^ bswap(tag[5])) |
                   (r1.z ^ bswap(tag[6])) | (r1.w ^ bswap(tag[7]));
        } else {
            const uint32_t items = ntok * nquads;
            // Items are taken 64 at a time from an LDS counter: the AES waves
            // that share a SIMD with a chain wave get fewer issue slots and so
            // take fewer items, and every SIMD finishes together (a static
            // stride left the chain SIMDs last: fused time = the sum of the
            // two sides).
            lds_word_t *next = (lds_word_t *)(uintptr_t)(DL2_FLAGS + 16u);
            for (;;) {
                uint32_t c0 = 0u;
                if (lane == 0u) c0 = __hip_atomic_fetch_add(next, 64u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                c0 = __builtin_amdgcn_readfirstlane(c0);
#ifdef RNSTOK_DL2_PROBE_SHA_ONLY
                break;
#endif
                if (c0 >= items) break;                 // wave-uniform
                // the tail chunk's idle lanes skip the body but stay in the
                // loop (a divergent `continue` let them re-enter the loop
                // head without lane 0 and spin on chunk 0: hang at n = 1)
                const uint32_t j = c0 + lane;
                if (j < items) {
                    const uint32_t t = base + j % ntok, q = j / ntok;
                    const uint32_t p = a.order ? a.order[t] : t;
                    const uint8_t *C = a.tok + in_off(a.tok_off, a.tok_stride, p) + 16 + 64ull * q;
                    uint8_t *D = a.pt + in_off(a.pt_off, a.pt_stride, p) + 64ull * q;
                    const uint32_t nbk = q + 1u == nquads ? tbl : 4u;
                    const u32x4 z = {0u, 0u, 0u, 0u};
                    u32x4 c[4], pp[4];
                    c[0] = ld16(C);
                    c[1] = nbk > 1 ? ld16(C + 16) : z;
                    c[2] = nbk > 2 ? ld16(C + 32) : z;
                    c[3] = nbk > 3 ? ld16(C + 48) : z;
                    const u32x4 chain = ld16(C - 16);      // previous ciphertext block (the IV for q = 0)
                    dec_quad_t01<NR>(pp, c, chain, K.rk, LN, inv_off);
                    st16(D, pp[0]);
                    if (nbk > 1) st16(D + 16, pp[1]);
                    if (nbk > 2) st16(D + 32, pp[2]);
                    if (nbk > 3) st16(D + 48, pp[3]);
                    if (q + 1u == nquads) {             // PKCS7.unpad's n = data[-1], for the chain wave
                        const u32x4 last = nbk == 1u ? pp[0] : (nbk == 2u ? pp[1] : (nbk == 3u ? pp[2] : pp[3]));
                        *(lds_word_t *)(uintptr_t)(DL2_PADN + 4u * (t - base)) = last.w >> 24;
                    }
                }
            }
        }
        __syncthreads();          // plaintext of every token of this batch is written; the ring is idle
        if (consumer) {
            const uint32_t t = base + slot_tok;
            if (slot_tok < ntok) {
                const uint32_t p = a.order ? a.order[t] : t;
                uint8_t *O = a.pt + in_off(a.pt_off, a.pt_stride, p);
                const uint32_t padn = *(lds_word_t *)(uintptr_t)(DL2_PADN + 4u * slot_tok);   // PKCS7.unpad: n = data[-1]
                const int32_t st = diff ? 2 : (padn > 16u ? 4 : 0);
                const uint32_t outlen = st == 0 ? 16u * nb - padn : (st == 4 ? padn : 0u);
                if (st != 0) {
                    const u32x4 z = {0u, 0u, 0u, 0u};
                    for (uint32_t i = 0; i < nb; ++i) st16(O + 16 * i, z);
                }
                a.status[p] = st;
                a.out_len[p] = outlen;
            }
        }
        if (threadIdx.x < 16u) tab_u32[(DL2_FLAGS >> 2) + threadIdx.x] = 0u;     // counters restart per batch
        __syncthreads();
    }
#ifndef RNSTOK_DL2_PROBE_AES_ONLY
    clk.finish(a.clk);
#endif
}

// --------------------------------------------------------- ratchet trials --
//
// Identity.decrypt (RNS/Identity.py:865-878) tries the receiver's ratchets in
// order and keeps the first whose derived token key opens the token (a wrong
// key raises in Token.decrypt and the loop moves on).  One lane per (token,
// candidate key) pair: HMAC-SHA256 over iv||ct under the candidate's
// midstates (Token.py:77-84), compared with the tag; the smallest matching
// rank per token wins (atomicMin).  A token that is not well-formed (len < 64
// or a ciphertext that is not whole blocks) never opens (Token.py:114), so it
// never matches.  The caller then decrypts each opened token with its key.
__global__ __launch_bounds__(256) void k_verify_trials(TrialArgs a) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= a.n_pairs) return;
    uint32_t lo = 0, hi = a.n_tok;             // token of pair j: last t with pair_off[t] <= j
    while (hi - lo > 1u) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a.pair_off[mid] <= j)
            lo = mid;
        else
            hi = mid;
    }
    const uint32_t t = lo, T = a.tok_len[t];
    if (T < 64u || ((T - 48u) & 15u)) return;
    const uint8_t *Kt = a.tok + a.tok_off[t];
    const uint32_t *r = a.rec + (uint64_t)a.pair_key[j] * REC_WORDS;
    uint32_t h[8], opad[8], tag[8];
    load8(h, r + REC_IPAD);
    const uint32_t M = T - 32u, full = M >> 6;
    for (uint32_t i = 0; i < full; ++i) {
        const uint8_t *B = Kt + 64ull * i;
        uint32_t w[16];
        sha_units(w, ld16(B), ld16(B + 16), ld16(B + 32), ld16(B + 48));
        sha256_compress(h, w);
    }
    const uint32_t fu = (M - 64u * full) >> 4;
    const uint8_t *R = Kt + 64ull * full;
    const u32x4 z = {0u, 0u, 0u, 0u};
    sha_final_units(h, fu, fu > 0 ? ld16(R) : z, fu > 1 ? ld16(R + 16) : z, fu > 2 ? ld16(R + 32) : z,
                    (uint64_t)(64u + M) * 8u);
    load8(opad, r + REC_OPAD);
    hmac_outer(tag, h, opad);
    const u32x4 r0 = ld16(Kt + M), r1 = ld16(Kt + M + 16);
    const uint32_t diff = (r0.x ^ bswap(tag[0])) | (r0.y ^ bswap(tag[1])) | (r0.z ^ bswap(tag[2])) |
                          (r0.w ^ bswap(tag[3])) | (r1.x ^ bswap(tag[4])) | (r1.y ^ bswap(tag[5])) |
                          (r1.z ^ bswap(tag[6])) | (r1.w ^ bswap(tag[7]));
    if (diff == 0u) atomicMin(a.first + t, j - a.pair_off[t]);
}

hipError_t launch_verify_trials(const TrialArgs &a, hipStream_t s) {
    hipError_t e = hipMemsetAsync(a.first, 0xFF, 4ull * a.n_tok, s);
    if (e != hipSuccess || a.n_pairs == 0) return e;
    hipLaunchKernelGGL(k_verify_trials, dim3((a.n_pairs + 255u) / 256u), dim3(256), 0, s, a);
    return hipGetLastError();
}

// ------------------------------------------------------------ verify_hmac --
//
// Token.verify_hmac (Token.py:77-84): HMAC-SHA256 over token[:-32] under the
// key's midstates, compared with token[-32:].  One lane per token; any length
// above 32 B (verify_hmac does not require whole AES blocks): full 64-B blocks
// from 16-B loads, the last partial block from 16-B units when it is whole
// units and from byte loads otherwise.  No AES runs and nothing but the status
// is written.

// rem (< 64) message bytes at p, then 0x80, zeros and the 64-bit length
// `bits`: the final one or two SHA-256 blocks, from byte loads.
__device__ __forceinline__ void sha_tail_bytes(uint32_t h[8], const uint8_t *p, uint32_t rem, uint64_t bits) {
    const uint32_t blocks = rem + 9u <= 64u ? 1u : 2u;
#pragma nounroll
    for (uint32_t b = 0; b < blocks; ++b) {
        uint32_t w[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            uint32_t v = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t q = 64u * b + 4u * k + j;
                v = (v << 8) | (q < rem ? (uint32_t)p[q] : (q == rem ? 0x80u : 0u));
            }
            w[k] = v;
        }
        if (b + 1u == blocks) {
            w[14] = (uint32_t)(bits >> 32);
            w[15] = (uint32_t)bits;
        }
        sha256_compress(h, w);
    }
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_verify(VerifyArgs a) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const uint32_t T = a.tok_len ? a.tok_len[i] : a.uni_len;
    if (T <= 32u) {                                   // Token.py:78
        a.status[i] = 1;
        return;
    }
    const uint8_t *Kt = a.tok + (a.tok_off ? a.tok_off[i] : (uint64_t)i * a.tok_stride);
    const uint32_t *r = a.rec + (a.key_idx ? (uint64_t)a.key_idx[i] * REC_WORDS : 0ull);
    uint32_t h[8], opad[8], tag[8];
    load8(h, r + REC_IPAD);
    const uint32_t M = T - 32u, full = M >> 6, rem = M & 63u;
    const uint64_t bits = (uint64_t)(64u + M) * 8u;
    for (uint32_t b = 0; b < full; ++b) {
        const uint8_t *B = Kt + 64ull * b;
        uint32_t w[16];
        sha_units(w, ld16(B), ld16(B + 16), ld16(B + 32), ld16(B + 48));
        sha256_compress(h, w);
    }
    const uint8_t *R = Kt + 64ull * full;
    if ((rem & 15u) == 0u) {                          // whole 16-B units (every well-formed token)
        const uint32_t fu = rem >> 4;
        const u32x4 z = {0u, 0u, 0u, 0u};
        sha_final_units(h, fu, fu > 0 ? ld16(R) : z, fu > 1 ? ld16(R + 16) : z, fu > 2 ? ld16(R + 32) : z, bits);
    } else {
        sha_tail_bytes(h, R, rem, bits);
    }
    load8(opad, r + REC_OPAD);
    hmac_outer(tag, h, opad);
    const u32x4 r0 = ld16(Kt + M), r1 = ld16(Kt + M + 16);
    const uint32_t diff = (r0.x ^ bswap(tag[0])) | (r0.y ^ bswap(tag[1])) | (r0.z ^ bswap(tag[2])) |
                          (r0.w ^ bswap(tag[3])) | (r1.x ^ bswap(tag[4])) | (r1.y ^ bswap(tag[5])) |
                          (r1.z ^ bswap(tag[6])) | (r1.w ^ bswap(tag[7]));
    a.status[i] = diff ? 2 : 0;                       // Token.py:82-84
}

hipError_t launch_verify(const VerifyArgs &a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_verify, dim3((a.n + 255u) / 256u), dim3(256), 0, s, a);
    return hipGetLastError();
}

// ------------------------------------------------------ length bucketing --
//
// Three small passes (histogram, scan, scatter) build a permutation that
// groups packets by descending quad count (64-B steps of the CBC/SHA loop).
// Per-workgroup LDS histograms keep global atomics to one per (workgroup,
// bucket).  Within a bucket the order is arbitrary.

__device__ __forceinline__ uint32_t sort_bucket(uint32_t len, int dec) {
    const uint32_t body = dec ? (len > 48u ? len - 48u : 0u) : len;
    const uint32_t q = body >> 6;
    return SORT_BUCKETS - 1u - (q < SORT_BUCKETS - 1u ? q : SORT_BUCKETS - 1u);   // descending
}

constexpr uint32_t SORT_TILE = 8192;   // packets per workgroup in the scatter pass

__global__ __launch_bounds__(1024) void k_sort_hist(const uint32_t *len, uint32_t n, int dec, uint32_t *hist) {
    __shared__ uint32_t h[SORT_BUCKETS];
    for (uint32_t b = threadIdx.x; b < SORT_BUCKETS; b += blockDim.x) h[b] = 0;
    __syncthreads();
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        atomicAdd(&h[sort_bucket(len[i], dec)], 1u);
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < SORT_BUCKETS; b += blockDim.x)
        if (h[b]) atomicAdd(&hist[b], h[b]);
}

__global__ __launch_bounds__(1024) void k_sort_scan(uint32_t *hist) {
    // exclusive scan of SORT_BUCKETS counters in place (one workgroup)
    __shared__ uint32_t part[1024];
    constexpr uint32_t PER = SORT_BUCKETS / 1024;
    uint32_t v[PER], sum = 0;
    for (uint32_t k = 0; k < PER; ++k) { v[k] = hist[threadIdx.x * PER + k]; sum += v[k]; }
    part[threadIdx.x] = sum;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {
        const uint32_t t = threadIdx.x >= off ? part[threadIdx.x - off] : 0u;
        __syncthreads();
        part[threadIdx.x] += t;
        __syncthreads();
    }
    uint32_t run = part[threadIdx.x] - sum;
    for (uint32_t k = 0; k < PER; ++k) { hist[threadIdx.x * PER + k] = run; run += v[k]; }
}

__global__ __launch_bounds__(1024) void k_sort_scatter(const uint32_t *len, uint32_t n, int dec, uint32_t *cursor,
                                                       uint32_t *order) {
    __shared__ uint32_t cnt[SORT_BUCKETS];
    __shared__ uint32_t base[SORT_BUCKETS];
    const uint32_t lo = blockIdx.x * SORT_TILE, hi = lo + SORT_TILE < n ? lo + SORT_TILE : n;
    for (uint32_t b = threadIdx.x; b < SORT_BUCKETS; b += blockDim.x) cnt[b] = 0;
    __syncthreads();
    for (uint32_t i = lo + threadIdx.x; i < hi; i += blockDim.x) atomicAdd(&cnt[sort_bucket(len[i], dec)], 1u);
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < SORT_BUCKETS; b += blockDim.x) {
        base[b] = cnt[b] ? atomicAdd(&cursor[b], cnt[b]) : 0u;
        cnt[b] = 0;
    }
    __syncthreads();
    for (uint32_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
        const uint32_t b = sort_bucket(len[i], dec);
        order[base[b] + atomicAdd(&cnt[b], 1u)] = i;
    }
}

uint64_t sort_workspace_bytes(uint32_t n) { return ((uint64_t)n * 4 + 255) / 256 * 256 + 2ull * SORT_BUCKETS * 4; }

hipError_t launch_length_order(const uint32_t *len, uint32_t n, int dec, void *workspace, const uint32_t **order,
                               uint32_t **queue, int n_cu, hipStream_t s) {
    uint32_t *ord = (uint32_t *)workspace;
    uint32_t *hist = (uint32_t *)((uint8_t *)workspace + ((uint64_t)n * 4 + 255) / 256 * 256);
    // hist[0..SORT_BUCKETS) and the chunk counter right after it, zeroed together
    hipError_t e = hipMemsetAsync(hist, 0, SORT_BUCKETS * 4 + 4, s);
    *queue = n <= QUEUE_MAX_N ? hist + SORT_BUCKETS : nullptr;   // past it: a static stride over the order
    if (e != hipSuccess) return e;
    const int gh = n_cu < (int)((n + 1023) / 1024) ? n_cu : (int)((n + 1023) / 1024);
    hipLaunchKernelGGL(k_sort_hist, dim3(gh > 0 ? gh : 1), dim3(1024), 0, s, len, n, dec, hist);
    hipLaunchKernelGGL(k_sort_scan, dim3(1), dim3(1024), 0, s, hist);
    hipLaunchKernelGGL(k_sort_scatter, dim3((n + SORT_TILE - 1) / SORT_TILE), dim3(1024), 0, s, len, n, dec, hist,
                       ord);
    *order = ord;
    return hipGetLastError();
}

// ------------------------------------------------------------- key setup --

// One lane per key, records staged through LDS (keysetup_device.h).
// NK = 8 (64-byte keys, AES-256) or 4 (32-byte keys, AES-128).
template <int NK>
__global__ __launch_bounds__(256) void k_key_setup(const uint8_t *keys, uint32_t n_keys, const uint8_t *sbox,
                                                    uint32_t *rec_out) {
    __shared__ uint8_t sb[256];
    __shared__ u32x4 stage[4][KS_STAGE_PIECES];
    sb[threadIdx.x] = sbox[threadIdx.x];          // blockDim.x == 256
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t kbase = blockIdx.x * blockDim.x + (wave << 6);
    const uint32_t k = kbase + lane < n_keys ? kbase + lane : n_keys - 1;   // tail lanes recompute the last key
    constexpr int HALF = 4 * NK;
    const uint8_t *key = keys + (uint64_t)k * (2 * HALF);
    const uint8_t *ek = key + HALF;                              // sk = key[:HALF], ek = key[HALF:]  (Token.py:61-70)
    uint32_t ekw[NK], skw[16];
#pragma unroll
    for (int i = 0; i < NK; ++i)
        ekw[i] = (uint32_t)ek[4 * i] | ((uint32_t)ek[4 * i + 1] << 8) | ((uint32_t)ek[4 * i + 2] << 16) |
                 ((uint32_t)ek[4 * i + 3] << 24);
#pragma unroll
    for (int i = 0; i < 16; ++i)
        skw[i] = 4 * i < HALF ? ((uint32_t)key[4 * i] << 24) | ((uint32_t)key[4 * i + 1] << 16) |
                                    ((uint32_t)key[4 * i + 2] << 8) | key[4 * i + 3]
                              : 0u;
    key_record<NK>(sb, ekw, skw, stage[wave], lane, kbase, n_keys, rec_out);
}

// --------------------------------------------------------------- launchers --

// Launch shape: a persistent grid of at most one workgroup per CU (the table
// image owns the CU's LDS).  Small batches (e.g. 16 KiB Resource tokens
// sharded 8 ways) shrink the workgroup instead of the grid so that every CU
// gets packets: threads = clamp(ceil(n / n_cu) rounded to a wave, 64, max).
struct Shape {
    int grid, threads;
};
static Shape shape_for(uint32_t n, int max_threads, int n_cu) {
    const uint64_t per_cu = ((uint64_t)n + n_cu - 1) / n_cu;
    uint64_t t = (per_cu + 63) / 64 * 64;
    if (t < 64) t = 64;
    if (t > (uint64_t)max_threads) t = max_threads;
    // Two passes per lane at most: split them evenly over whole sets of 4
    // waves (e.g. 2^18 packets at 768 threads gave a third of the lanes a
    // second packet and doubled a latency-bound launch; 512 threads x 2 do
    // not).  Longer batches keep the widest shape and balance by chunks.
    if (per_cu > (uint64_t)max_threads && per_cu <= 2ull * (uint64_t)max_threads) {
        const uint64_t half = (per_cu + 1) / 2;
        t = (half + 255) / 256 * 256;
        if (t > (uint64_t)max_threads) t = max_threads;
    }
    uint64_t g = ((uint64_t)n + t - 1) / t;
    if (g > (uint64_t)n_cu) g = n_cu;
    if (g < 1) g = 1;
#ifndef RNSTOK_NO_SMALL_FILL
    // One workgroup (up to 64 packets, e.g. a single Token.encrypt): widen it
    // so the LDS table image is written by 512 threads, not 64 (the extra
    // waves find no packet and leave after fill_tables).
    if (g == 1 && t < 512 && max_threads >= 512) t = 512;
#endif
    return {(int)g, (int)t};
}

#ifndef RNSTOK_SPLIT_ENC            // 0: every single-key uniform batch on k_encrypt (the A/B baseline)
#define RNSTOK_SPLIT_ENC 1
#endif
#ifndef RNSTOK_SPLIT_ROWS_RB          // packed rows: LDS ring (0) or read-back (1)
#define RNSTOK_SPLIT_ROWS_RB 0
#endif
#ifndef RNSTOK_SPLIT_ILV_RB           // interleaved: read-back (1) or LDS ring (0)
#define RNSTOK_SPLIT_ILV_RB 1
#endif
// Split-role encrypt (k_encrypt_split): uniform lengths, at least one
// 64-packet batch per AES wave of every CU.
#ifndef RNSTOK_SPLIT_PERKEY          // per-packet keys (c3) on the split kernel too: 0.845 vs 0.912 ms rows,
#define RNSTOK_SPLIT_PERKEY 1        // 0.770 vs 0.852 interleaved (profiles/r04_split/r04i_perkey_ab.txt)
#endif
#ifndef RNSTOK_SPLIT_GEN             // packed / length-ordered batches (c5) on the split kernel too
#define RNSTOK_SPLIT_GEN 1
#endif
static bool use_split_enc(const EncArgs &a, int n_cu) {
    const bool gen = a.pt_len || a.order || a.queue || a.pt_off;
    return RNSTOK_SPLIT_ENC && (!a.key_idx || RNSTOK_SPLIT_PERKEY) && (!gen || RNSTOK_SPLIT_GEN) &&
           (uint64_t)a.n >= 64ull * SPLIT_AES_WAVES * (uint64_t)n_cu;
}
static uint64_t split_grid(uint32_t n, int n_cu) {
    const uint64_t batches = (n + 63ull) / 64ull;
    uint64_t grid = (batches + SPLIT_AES_WAVES - 1) / SPLIT_AES_WAVES;
    return grid > (uint64_t)n_cu ? (uint64_t)n_cu : grid;
}
template <int NR>
static hipError_t launch_enc_split_nr(const EncArgs &a, int n_cu, hipStream_t s) {
    const uint64_t grid = split_grid(a.n, n_cu);
#define RT_SPLIT(ILV_, RB_, PK_, GEN_)                                                                        \
    hipLaunchKernelGGL((k_encrypt_split<NR, ILV_, RB_, PK_, GEN_>), dim3((unsigned)grid), dim3(SPLIT_THREADS), \
                       LDS_ENC_SPLIT_BYTES, s, a)
    const bool gen = a.pt_len || a.order || a.queue || a.pt_off;
    if (gen && a.key_idx)
        RT_SPLIT(false, false, true, true);
    else if (gen)
        RT_SPLIT(false, false, false, true);
    else if (a.ilv && a.key_idx)
        RT_SPLIT(true, RNSTOK_SPLIT_ILV_RB, true, false);
    else if (a.ilv)
        RT_SPLIT(true, RNSTOK_SPLIT_ILV_RB, false, false);
    else if (a.key_idx)
        RT_SPLIT(false, RNSTOK_SPLIT_ROWS_RB, true, false);
    else
        RT_SPLIT(false, RNSTOK_SPLIT_ROWS_RB, false, false);
#undef RT_SPLIT
    return hipGetLastError();
}

template <int NR>
static hipError_t launch_enc_nr(const EncArgs &a, Shape sh, hipStream_t s) {
    if (a.ilv && a.key_idx)
        hipLaunchKernelGGL((k_encrypt<NR, true, true>), dim3(sh.grid), dim3(sh.threads), LDS_ENC_BYTES, s, a);
    else if (a.ilv)
        hipLaunchKernelGGL((k_encrypt<NR, false, true>), dim3(sh.grid), dim3(sh.threads), LDS_ENC_BYTES, s, a);
    else if (a.key_idx)
        hipLaunchKernelGGL((k_encrypt<NR, true>), dim3(sh.grid), dim3(sh.threads), LDS_ENC_BYTES, s, a);
    else
        hipLaunchKernelGGL((k_encrypt<NR, false>), dim3(sh.grid), dim3(sh.threads), LDS_ENC_BYTES, s, a);
    return hipGetLastError();
}
template <int NR>
static hipError_t launch_dec_nr(const DecArgs &a, Shape sh, hipStream_t s) {
    if (a.ilv && a.key_idx)
        hipLaunchKernelGGL((k_decrypt<NR, true, WG_PERKEY_DEC, true>), dim3(sh.grid), dim3(sh.threads), LDS_DEC_BYTES,
                           s, a);
    else if (a.ilv && sh.threads > WG_DEC)
        hipLaunchKernelGGL((k_decrypt<NR, false, 1024, true>), dim3(sh.grid), dim3(sh.threads), LDS_DEC_BYTES, s, a);
    else if (a.ilv)
        hipLaunchKernelGGL((k_decrypt<NR, false, WG_DEC, true>), dim3(sh.grid), dim3(sh.threads), LDS_DEC_BYTES, s, a);
    else if (a.key_idx)
        hipLaunchKernelGGL((k_decrypt<NR, true>), dim3(sh.grid), dim3(sh.threads), LDS_DEC_BYTES, s, a);
    else if (sh.threads > WG_DEC)
        hipLaunchKernelGGL((k_decrypt<NR, false, 1024>), dim3(sh.grid), dim3(sh.threads), LDS_DEC_BYTES, s, a);
    else
        hipLaunchKernelGGL((k_decrypt<NR, false>), dim3(sh.grid), dim3(sh.threads), LDS_DEC_BYTES, s, a);
    return hipGetLastError();
}

template <int NR>
static hipError_t launch_enc_long_nr(const EncArgs &a, int n_cu, hipStream_t s) {
    const uint32_t G = a.n > 64u * (uint32_t)n_cu ? 2u : 1u;          // token groups of 64 per workgroup
    uint64_t grid = (a.n + 64ull * G - 1) / (64ull * G);
    if (grid > (uint64_t)n_cu) grid = n_cu;
    if (a.key_idx)
        hipLaunchKernelGGL((k_encrypt_long<NR, true>), dim3((unsigned)grid), dim3(128 * G), LDS_ENC_LONG_BYTES, s, a);
    else
        hipLaunchKernelGGL((k_encrypt_long<NR, false>), dim3((unsigned)grid), dim3(128 * G), LDS_ENC_LONG_BYTES, s, a);
    return hipGetLastError();
}

// Long-token mode: uniform batches that give each CU at most two waves of
// packets in the one-lane-per-packet kernel, where each lane's serial chain
// (one instruction per ~4 cycles from a wave that has its SIMD nearly to
// itself) is the whole launch.  The single-key kernels (k_encrypt_long4,
// k_decrypt_long2) split every chain over lanes and waves and win at every
// length there (2^15 x 500 B: encrypt 103 -> 58 us, decrypt 105 -> 49 us;
// one 500-B packet: 91 -> 51 and 113 -> 34 us; profiles/r02v_lat.txt), so
// they take any length.  So does the per-key k_encrypt_long (2^15 x 500 B
// with 64 keys: 101 -> 80 us; x 1000 B: 172 -> 129 us; even at 100 B;
// profiles/r02x_lat_perkey.txt).
#ifndef RNSTOK_LONG_MIN_LEN
#define RNSTOK_LONG_MIN_LEN 0u
#endif
#ifndef RNSTOK_LONG_PERKEY_MIN_LEN
#define RNSTOK_LONG_PERKEY_MIN_LEN 0u
#endif
// Tokens per CU up to which the long-token kernels run (one persistent
// workgroup of 128 chains per CU).  A build with a larger value forces them
// onto big batches: the measured comparison of their lane-cooperative CBC
// and wave-split HMAC with one packet per lane at c2.
#ifndef RNSTOK_LONG_MAX_PER_CU
#define RNSTOK_LONG_MAX_PER_CU 128ull
#endif
static bool use_long(uint32_t n, const uint32_t *len, uint32_t uni, int n_cu, uint32_t min_len) {
    return len == nullptr && uni >= min_len && (uint64_t)n <= RNSTOK_LONG_MAX_PER_CU * (uint64_t)n_cu;
}

template <int NR>
static hipError_t launch_enc_long4_nr(const EncArgs &a, int n_cu, hipStream_t s) {
    uint64_t grid = (a.n + L4_TOK - 1ull) / L4_TOK;
    if (grid > (uint64_t)n_cu) grid = n_cu;
    hipLaunchKernelGGL((k_encrypt_long4<NR>), dim3((unsigned)grid), dim3(L4_THREADS), LDS_ENC_LONG4_BYTES, s, a);
    return hipGetLastError();
}

// A uniform batch whose packets do not divide evenly over the persistent
// grid's lanes (e.g. 2^20 packets over 256 x 768 per-packet-key lanes: 5.33
// per lane) would leave a third of the workgroups one packet longer; there
// the dynamic chunk loop balances the SIMDs instead.
template <class Args>
static hipError_t balance(Args &a, Shape sh, SpareQueue *spare, hipStream_t s, bool *took, uint32_t *slot) {
    const uint64_t lanes = (uint64_t)sh.grid * (uint64_t)sh.threads;
    *took = false;
    // (whole passes keep the static stride: the counter measured -4..-7 % at
    // 5 and 6 passes but +2.3 % at 4 on two boxes, profiles/r05h_dyn/)
    if (a.queue || !spare || a.n <= lanes || a.n % lanes == 0 || a.n > QUEUE_MAX_N) return hipSuccess;
    a.queue = spare->acquire(s, slot);
    if (!a.queue) return hipSuccess;     // no slot: the static stride (correct, less balanced)
    *took = true;
    return hipMemsetAsync(a.queue, 0, 4, s);
}

int plan_encrypt(uint32_t n, bool packed, uint32_t uni_len, bool per_key, int n_cu) {
    const uint32_t *len = packed ? &uni_len : nullptr;   // any non-null marks a packed batch
#ifndef RNSTOK_NO_LONG4
    if (!per_key && use_long(n, len, uni_len, n_cu, RNSTOK_LONG_MIN_LEN)) return RT_KERNEL_ENC_LONG4;
#endif
    if (use_long(n, len, uni_len, n_cu, RNSTOK_LONG_PERKEY_MIN_LEN)) return RT_KERNEL_ENC_LONG;
    EncArgs a{};
    a.n = n; a.uni_len = uni_len; a.pt_len = len; a.key_idx = per_key ? &uni_len : nullptr;
    if (use_split_enc(a, n_cu)) return RT_KERNEL_ENC_SPLIT;
    return RT_KERNEL_GENERAL;
}

hipError_t launch_encrypt(const EncArgs &args, int nr, int n_cu, SpareQueue *spare, hipStream_t s) {
    EncArgs a = args;
    const int plan = a.ilv ? RT_KERNEL_GENERAL : plan_encrypt(a.n, a.pt_len != nullptr, a.uni_len, a.key_idx != nullptr, n_cu);
    if (plan == RT_KERNEL_ENC_LONG4)
        return nr == 14 ? launch_enc_long4_nr<14>(a, n_cu, s) : launch_enc_long4_nr<10>(a, n_cu, s);
    if (plan == RT_KERNEL_ENC_LONG)
        return nr == 14 ? launch_enc_long_nr<14>(a, n_cu, s) : launch_enc_long_nr<10>(a, n_cu, s);

    if (use_split_enc(a, n_cu)) {
        // Uniform row batches that do not give every AES wave the same number
        // of 64-packet batches take them from a chunk counter instead of the
        // static stride, as k_decrypt's ragged batches do (balance): 2^20 x
        // 500 B (8 per AES wave) keeps the stride; 983 040 x 500 B (7.5 per
        // wave) -4.8..-5.8 %, 1.5 M x 500 B -4.6..-10 % on three boxes
        // (profiles/r05h_dyn/).  Short packets keep the stride: a counter
        // fetch is an L2 round trip per batch, +18 % at 100 B.
        const bool gen = a.pt_len || a.order || a.queue || a.pt_off;
        const uint64_t waves = split_grid(a.n, n_cu) * SPLIT_AES_WAVES, batches = (a.n + 63ull) / 64ull;
        bool took = false;
        uint32_t slot = 0;
        if (RNSTOK_SPLIT_DYN && !gen && !a.ilv && spare && a.n <= QUEUE_MAX_N && batches % waves != 0 &&
            a.uni_len >= RNSTOK_SPLIT_DYN_MIN_LEN) {
            a.queue = spare->acquire(s, &slot);
            took = a.queue != nullptr;
            if (took) {
                hipError_t e = hipMemsetAsync(a.queue, 0, 4, s);
                if (e != hipSuccess) {
                    spare->release(s, slot);
                    return e;
                }
            }
        }
        hipError_t e = nr == 14 ? launch_enc_split_nr<14>(a, n_cu, s) : launch_enc_split_nr<10>(a, n_cu, s);
        if (took) spare->release(s, slot);
        return e;
    }
    const Shape sh = shape_for(a.n, a.key_idx ? WG_PERKEY_ENC : WG_ENC, n_cu);
    bool took = false;
    uint32_t slot = 0;
    hipError_t e = balance(a, sh, spare, s, &took, &slot);
    if (e == hipSuccess) e = nr == 14 ? launch_enc_nr<14>(a, sh, s) : launch_enc_nr<10>(a, sh, s);
    if (took) spare->release(s, slot);
    return e;
}
template <int NR>
static hipError_t launch_dec_long_nr(const DecArgs &a, int n_cu, hipStream_t s) {
    uint64_t grid = (a.n + 127ull) / 128ull;
    if (grid > (uint64_t)n_cu) grid = n_cu;
    hipLaunchKernelGGL((k_decrypt_long2<NR>), dim3((unsigned)grid), dim3(DL2_THREADS), LDS_DL2_BYTES, s, a);
    return hipGetLastError();
}

int plan_decrypt(uint32_t n, bool packed, uint32_t uni_len, bool per_key, int n_cu) {
    // long mode: one key, uniform well-formed tokens (whole blocks, at least
    // one), few per CU
    if (!per_key && !packed && uni_len >= 64u && uni_len >= 48u + RNSTOK_LONG_MIN_LEN &&
        ((uni_len - 48u) & 15u) == 0 && (uint64_t)n <= RNSTOK_LONG_MAX_PER_CU * (uint64_t)n_cu)
        return RT_KERNEL_DEC_LONG2;
    return RT_KERNEL_GENERAL;
}

hipError_t launch_decrypt(const DecArgs &args, int nr, int n_cu, SpareQueue *spare, hipStream_t s) {
    DecArgs a = args;
    if (!a.ilv && plan_decrypt(a.n, a.tok_len != nullptr, a.uni_len, a.key_idx != nullptr, n_cu) == RT_KERNEL_DEC_LONG2)
        return nr == 14 ? launch_dec_long_nr<14>(a, n_cu, s) : launch_dec_long_nr<10>(a, n_cu, s);
    // one key and one pass at up to 1024 threads: the 1024-thread instance;
    // so do uniform short tokens (4 waves/SIMD cover the per-token hash tail
    // and loads, which the 768-thread instance's pairing does not pay for:
    // 2^20 tokens of 16-250 B plaintext -8..-31 %, 350-430 B +1..+2 %,
    // profiles/r05r_short/)
    const uint64_t per_cu = ((uint64_t)a.n + n_cu - 1) / n_cu;
    const bool short_tok = !a.tok_len && a.uni_len <= RNSTOK_DEC1024_MAX_TOKEN;
    const int max_t = a.key_idx ? WG_PERKEY_DEC : ((per_cu <= 1024u || short_tok) ? 1024 : WG_DEC);
    const Shape sh = shape_for(a.n, max_t, n_cu);
    bool took = false;
    uint32_t slot = 0;
    hipError_t e = balance(a, sh, spare, s, &took, &slot);
    if (e == hipSuccess) e = nr == 14 ? launch_dec_nr<14>(a, sh, s) : launch_dec_nr<10>(a, sh, s);
    if (took) spare->release(s, slot);
    return e;
}
hipError_t launch_key_setup(const uint8_t *keys, uint32_t key_len, uint32_t n_keys, const uint8_t *sbox,
                            uint32_t *rec, hipStream_t s) {
    if (key_len == 64)
        hipLaunchKernelGGL(k_key_setup<8>, dim3((n_keys + 255) / 256), dim3(256), 0, s, keys, n_keys, sbox, rec);
    else
        hipLaunchKernelGGL(k_key_setup<4>, dim3((n_keys + 255) / 256), dim3(256), 0, s, keys, n_keys, sbox, rec);
    return hipGetLastError();
}
hipError_t configure_kernels() {
    // 128 / 160 KiB of dynamic LDS per workgroup is above the default cap.
    hipError_t e = hipSuccess;
#define RT_CFG(k, bytes)                                                                                     \
    if (e == hipSuccess) e = hipFuncSetAttribute((const void *)(k), hipFuncAttributeMaxDynamicSharedMemorySize, \
                                                 (int)(bytes))
    RT_CFG((k_encrypt<14, false>), LDS_ENC_BYTES);
    RT_CFG((k_encrypt<14, true>), LDS_ENC_BYTES);
    RT_CFG((k_encrypt<10, false>), LDS_ENC_BYTES);
    RT_CFG((k_encrypt<10, true>), LDS_ENC_BYTES);
    RT_CFG((k_decrypt_long2<14>), LDS_DL2_BYTES);
    RT_CFG((k_decrypt_long2<10>), LDS_DL2_BYTES);
    RT_CFG((k_encrypt_long4<14>), LDS_ENC_LONG4_BYTES);
    RT_CFG((k_encrypt_long4<10>), LDS_ENC_LONG4_BYTES);
    RT_CFG((k_encrypt_long<14, false>), LDS_ENC_LONG_BYTES);
    RT_CFG((k_encrypt_long<14, true>), LDS_ENC_LONG_BYTES);
    RT_CFG((k_encrypt_long<10, false>), LDS_ENC_LONG_BYTES);
    RT_CFG((k_encrypt_long<10, true>), LDS_ENC_LONG_BYTES);
    RT_CFG((k_decrypt<14, false>), LDS_DEC_BYTES);
    RT_CFG((k_decrypt<14, false, 1024>), LDS_DEC_BYTES);
    RT_CFG((k_decrypt<14, true>), LDS_DEC_BYTES);
    RT_CFG((k_decrypt<10, false>), LDS_DEC_BYTES);
    RT_CFG((k_decrypt<10, false, 1024>), LDS_DEC_BYTES);
    RT_CFG((k_decrypt<10, true>), LDS_DEC_BYTES);
    RT_CFG((k_encrypt<14, false, true>), LDS_ENC_BYTES);
    RT_CFG((k_encrypt<14, true, true>), LDS_ENC_BYTES);
    RT_CFG((k_encrypt<10, false, true>), LDS_ENC_BYTES);
    RT_CFG((k_encrypt<10, true, true>), LDS_ENC_BYTES);
    RT_CFG((k_decrypt<14, false, WG_DEC, true>), LDS_DEC_BYTES);
    RT_CFG((k_decrypt<14, false, 1024, true>), LDS_DEC_BYTES);
    RT_CFG((k_decrypt<14, true, WG_PERKEY_DEC, true>), LDS_DEC_BYTES);
    RT_CFG((k_decrypt<10, false, WG_DEC, true>), LDS_DEC_BYTES);
    RT_CFG((k_decrypt<10, false, 1024, true>), LDS_DEC_BYTES);
    RT_CFG((k_decrypt<10, true, WG_PERKEY_DEC, true>), LDS_DEC_BYTES);
    RT_CFG((k_encrypt_split<14, false, false, false, true>), LDS_ENC_SPLIT_BYTES);
    RT_CFG((k_encrypt_split<14, false, false, true, true>), LDS_ENC_SPLIT_BYTES);
    RT_CFG((k_encrypt_split<10, false, false, false, true>), LDS_ENC_SPLIT_BYTES);
    RT_CFG((k_encrypt_split<10, false, false, true, true>), LDS_ENC_SPLIT_BYTES);
    RT_CFG((k_encrypt_split<14, false, RNSTOK_SPLIT_ROWS_RB, false>), LDS_ENC_SPLIT_BYTES);
    RT_CFG((k_encrypt_split<14, true, RNSTOK_SPLIT_ILV_RB, false>), LDS_ENC_SPLIT_BYTES);
    RT_CFG((k_encrypt_split<10, false, RNSTOK_SPLIT_ROWS_RB, false>), LDS_ENC_SPLIT_BYTES);
    RT_CFG((k_encrypt_split<10, true, RNSTOK_SPLIT_ILV_RB, false>), LDS_ENC_SPLIT_BYTES);
    RT_CFG((k_encrypt_split<14, false, RNSTOK_SPLIT_ROWS_RB, true>), LDS_ENC_SPLIT_BYTES);
    RT_CFG((k_encrypt_split<14, true, RNSTOK_SPLIT_ILV_RB, true>), LDS_ENC_SPLIT_BYTES);
    RT_CFG((k_encrypt_split<10, false, RNSTOK_SPLIT_ROWS_RB, true>), LDS_ENC_SPLIT_BYTES);
    RT_CFG((k_encrypt_split<10, true, RNSTOK_SPLIT_ILV_RB, true>), LDS_ENC_SPLIT_BYTES);
#undef RT_CFG
    return e;
}

}  // namespace rnstok

#ifdef RNSTOK_SPLIT_PROBE
// probe builds only: read and clear k_encrypt_split's wait counters
extern "C" int rt_split_probe_read(unsigned long long *out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(rnstok::g_split_probe), sizeof(unsigned long long) * 8) != hipSuccess)
        return -1;
    const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    return hipMemcpyToSymbol(HIP_SYMBOL(rnstok::g_split_probe), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
