// hkdf_kernels.hip — batched HKDF-SHA256 (RNS/Cryptography/HKDF.py:35-62).
//
// Identity.encrypt / __decrypt derive a fresh 64-byte token key per packet
// (Identity.py:837-846, salt = the identity hash, context None) and
// Link.handshake one per link; the derived keys feed Token(key).  Here one
// lane derives one key: the salt becomes the HMAC key (HMAC.py:73-82: zero
// padded to 64 bytes, hashed first when longer), PRK = HMAC(salt, ikm), then
// T_i = HMAC(PRK, T_{i-1} || context || i mod 256) with the PRK's ipad/opad
// midstates computed once.  With 32-byte ikm, 16-byte salt, no context and a
// 64-byte output that is 10 SHA-256 compressions per lane.
//
// The generic instance assembles the messages word by word from byte loads
// (global memory is read once per byte; the previous block T_{i-1} comes from
// registers), so any lengths work.  The common shape (ikm and salt whole
// 4-byte words, ikm <= 52 bytes so PRK's message is one block, no context)
// takes the FAST instance: dword loads and the padded blocks written as
// constants.  Both are VALU-bound like the token MAC.
#include "keysetup_device.h"
#include "token_device.h"
#include "token_launch.h"

namespace rnstok {

namespace {

__device__ const uint32_t SHA_IV[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                       0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

// Byte q of  seg[0..seg_len) || tail (if tail >= 0) || 0x80 || zeros.
__device__ __forceinline__ uint32_t msg_byte(const uint8_t *seg, uint32_t seg_len, int tail, uint32_t q) {
    const uint32_t body = seg_len + (tail >= 0 ? 1u : 0u);
    if (q < seg_len) return seg[q];
    if (q < body) return (uint32_t)tail;
    return q == body ? 0x80u : 0u;
}

// SHA-256 of  pre[0..npre) words || seg || tail  appended to `prior` bytes
// already absorbed into h (prior = 64 after an HMAC ipad/opad block), with
// the final padding.  npre is 0 or 8 (the previous HKDF block).
__device__ __forceinline__ void sha_msg(uint32_t h[8], uint32_t prior, const uint32_t pre[8], uint32_t npre,
                                     const uint8_t *seg, uint32_t seg_len, int tail) {
    const uint64_t m = 4ull * npre + seg_len + (tail >= 0 ? 1u : 0u);
    const uint64_t bits = (prior + m) * 8ull;
    const uint64_t nblk = (m + 8u) / 64u + 1u;
    for (uint64_t b = 0; b < nblk; ++b) {
        uint32_t w[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if (b == 0 && (uint32_t)k < npre) {
                w[k] = pre[k];
            } else {
                const uint32_t q = (uint32_t)(64u * b + 4u * k) - 4u * npre;
                w[k] = (msg_byte(seg, seg_len, tail, q) << 24) | (msg_byte(seg, seg_len, tail, q + 1) << 16) |
                       (msg_byte(seg, seg_len, tail, q + 2) << 8) | msg_byte(seg, seg_len, tail, q + 3);
            }
        }
        if (b + 1 == nblk) {
            w[14] = (uint32_t)(bits >> 32);
            w[15] = (uint32_t)bits;
        }
        sha256_compress(h, w);
    }
}

// HMAC ipad / opad midstates for a key (HMAC.py:73-82).
__device__ __forceinline__ void hmac_midstates(const uint32_t key[16], uint32_t hi[8], uint32_t ho[8]) {
    uint32_t wi[16], wo[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        wi[i] = key[i] ^ 0x36363636u;
        wo[i] = key[i] ^ 0x5c5c5c5cu;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) hi[i] = ho[i] = SHA_IV[i];
    sha256_compress(hi, wi);
    sha256_compress(ho, wo);
}

// The same, one compression at a time (no interleaving of the two chains:
// register pressure in k_hkdf_key_setup).
__device__ __forceinline__ void hmac_midstates_serial(const uint32_t key[16], uint32_t hi[8], uint32_t ho[8]) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = key[i] ^ 0x36363636u;
#pragma unroll
    for (int i = 0; i < 8; ++i) hi[i] = ho[i] = SHA_IV[i];
    sha256_compress_fenced(hi, w);
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = key[i] ^ 0x5c5c5c5cu;
    sha256_compress_fenced(ho, w);
}

__device__ __forceinline__ void hmac_outer_fenced(uint32_t tag[8], const uint32_t inner[8], const uint32_t opad[8]) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) { w[i] = inner[i]; tag[i] = opad[i]; }
    w[8] = 0x80000000u;
#pragma unroll
    for (int i = 9; i < 15; ++i) w[i] = 0;
    w[15] = (64 + 32) * 8;
    sha256_compress_fenced(tag, w);
}

// big-endian word at a 4-byte aligned address (FAST instance only)
__device__ __forceinline__ uint32_t ld_be32(const uint8_t *p) {
    return bswap(*(const uint32_t *)__builtin_assume_aligned(p, 4));
}

// HMAC(salt, .) ipad / opad midstates for key row i.
template <bool FAST, bool FENCED = false>
__device__ __forceinline__ void salt_midstates(const HkdfArgs &a, uint64_t i, uint32_t hi[8], uint32_t ho[8]) {
    // HMAC key = salt; None / empty salt -> 32 zero bytes (HKDF.py:45-46), which
    // zero-pads to the same 64-byte block as an empty key.
    uint32_t key[16];
    const uint32_t sl = a.salt ? a.salt_len : 0u;
    const uint8_t *salt = a.salt ? a.salt + i * a.salt_stride : nullptr;
    if (FAST) {                                       // sl % 4 == 0, sl <= 64
#pragma unroll
        for (int k = 0; k < 16; ++k) key[k] = 4u * k < sl ? ld_be32(salt + 4 * k) : 0u;
    } else if (sl > 64u) {                            // HMAC.py: long keys are hashed first
        uint32_t d[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) d[k] = SHA_IV[k];
        sha_msg(d, 0u, nullptr, 0u, salt, sl, -1);
#pragma unroll
        for (int k = 0; k < 16; ++k) key[k] = k < 8 ? d[k] : 0u;
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            uint32_t v = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t q = 4u * k + j;
                v = (v << 8) | (q < sl ? salt[q] : 0u);
            }
            key[k] = v;
        }
    }
    if (FENCED)
        hmac_midstates_serial(key, hi, ho);
    else
        hmac_midstates(key, hi, ho);
}

// SHARED: one salt row for every key (salt_stride 0: a batch to one identity,
// Identity.py:837-846, salt = the identity hash).  Its midstates are then
// computed once per lane and reused over the lane's keys (grid-stride loop).
template <bool FAST, bool SHARED>
__global__ __launch_bounds__(256) void k_hkdf(HkdfArgs a) {
    const uint64_t first = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t step = SHARED ? (uint64_t)gridDim.x * blockDim.x : (uint64_t)a.n;   // else one key per lane
    if (first >= a.n) return;
    uint32_t shi[8], sho[8];
    if (SHARED) salt_midstates<FAST>(a, 0, shi, sho);
    for (uint64_t i = first; i < a.n; i += step) {
        const uint8_t *ikm = a.ikm + i * a.ikm_stride;
        uint32_t hi[8], ho[8], inner[8], prk[8];
        if (SHARED) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                hi[k] = shi[k];
                ho[k] = sho[k];
            }
        } else {
            salt_midstates<FAST>(a, i, hi, ho);
        }
        uint32_t key[16];
#pragma unroll
        for (int k = 0; k < 8; ++k) inner[k] = hi[k];
        if (FAST) {                                       // ikm_len % 4 == 0, ikm_len <= 52: one block
            uint32_t w[16];
#pragma unroll
            for (int k = 0; k < 14; ++k)
                w[k] = 4u * k < a.ikm_len ? ld_be32(ikm + 4 * k) : (4u * k == a.ikm_len ? 0x80000000u : 0u);
            w[14] = 0u;
            w[15] = (64u + a.ikm_len) * 8u;
            sha256_compress(inner, w);
        } else {
            sha_msg(inner, 64u, nullptr, 0u, ikm, a.ikm_len, -1);
        }
        hmac_outer(prk, inner, ho);                      // PRK = HMAC(salt, ikm)  (HKDF.py:51)
#pragma unroll
        for (int k = 0; k < 16; ++k) key[k] = k < 8 ? prk[k] : 0u;
        hmac_midstates(key, hi, ho);
        uint32_t t[8];
        uint8_t *out = a.out + (uint64_t)i * a.out_stride;
        for (uint32_t blk = 0, done = 0; done < a.length; ++blk) {
#pragma unroll
            for (int k = 0; k < 8; ++k) inner[k] = hi[k];
            // T_blk = HMAC(PRK, T_{blk-1} || context || (blk+1) % 256)  (HKDF.py:56-60)
            if (FAST) {                                   // T_{blk-1} (32 B, none for blk 0) || counter byte
                const uint32_t ctr = (((blk + 1u) & 255u) << 24) | 0x00800000u;
                uint32_t w[16];
#pragma unroll
                for (int k = 0; k < 16; ++k) w[k] = 0u;
                if (blk) {
#pragma unroll
                    for (int k = 0; k < 8; ++k) w[k] = t[k];
                    w[8] = ctr;
                    w[15] = (64u + 33u) * 8u;
                } else {
                    w[0] = ctr;
                    w[15] = (64u + 1u) * 8u;
                }
                sha256_compress(inner, w);
            } else {
                sha_msg(inner, 64u, t, blk ? 8u : 0u, a.context, a.context_len, (int)((blk + 1u) & 255u));
            }
            hmac_outer(t, inner, ho);
            const uint32_t take = a.length - done < 32u ? a.length - done : 32u;
            if (take == 32u) {
                st16(out + done, u32x4{bswap(t[0]), bswap(t[1]), bswap(t[2]), bswap(t[3])});
                st16(out + done + 16, u32x4{bswap(t[4]), bswap(t[5]), bswap(t[6]), bswap(t[7])});
            } else {
                for (uint32_t j = 0; j < take; ++j) {
                    uint32_t wv = t[0];
#pragma unroll
                    for (int k = 1; k < 8; ++k)
                        if ((j >> 2) == (uint32_t)k) wv = t[k];
                    out[done + j] = (uint8_t)(wv >> (24u - 8u * (j & 3u)));
                }
            }
            done += take;
        }
    }
}

// HKDF and key setup fused (the FAST shape: no context, ikm <= 52 B and salt
// <= 64 B in whole aligned words): per-packet keying as Identity.encrypt /
// __decrypt construct it (Identity.py:837-846, Token(hkdf(64, shared_key,
// salt))).  Each lane derives its key into registers — T1 (and T2 for 64-B
// keys) — and builds its record exactly as k_key_setup does from memory, so
// the derived keys never reach HBM and one launch replaces two.  The loop is
// wave-uniform (records are staged per wave); SHARED keeps the salt's
// midstates for the lane's keys.
template <bool SHARED, int NK>
// 3 waves per SIMD: the 48 KiB staging area admits 3 workgroups per CU
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void k_hkdf_key_setup(HkdfArgs a, const uint8_t *sbox, uint32_t *rec_out) {
    __shared__ uint8_t sb[256];
    __shared__ u32x4 stage[4][KS_STAGE_PIECES];
    sb[threadIdx.x] = sbox[threadIdx.x];          // blockDim.x == 256
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint32_t shi[8], sho[8];
    if (SHARED) salt_midstates<true, true>(a, 0, shi, sho);
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t kb = (uint64_t)blockIdx.x * blockDim.x + (wave << 6); kb < a.n; kb += step) {
        const uint32_t kbase = (uint32_t)kb;
        const uint32_t i = kbase + lane < a.n ? kbase + lane : a.n - 1u;   // tail lanes: a copy of the last key
        uint32_t hi[8], ho[8], inner[8], prk[8];
        if (SHARED) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                hi[k] = shi[k];
                ho[k] = sho[k];
            }
        } else {
            salt_midstates<true, true>(a, i, hi, ho);
        }
        const uint8_t *ikm = a.ikm + (uint64_t)i * a.ikm_stride;
        {
            uint32_t w[16];
#pragma unroll
            for (int k = 0; k < 14; ++k)
                w[k] = 4u * k < a.ikm_len ? ld_be32(ikm + 4 * k) : (4u * k == a.ikm_len ? 0x80000000u : 0u);
            w[14] = 0u;
            w[15] = (64u + a.ikm_len) * 8u;
#pragma unroll
            for (int k = 0; k < 8; ++k) inner[k] = hi[k];
            sha256_compress_fenced(inner, w);
        }
        hmac_outer_fenced(prk, inner, ho);                      // PRK = HMAC(salt, ikm)  (HKDF.py:51)
        {
            uint32_t key[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) key[k] = k < 8 ? prk[k] : 0u;
            hmac_midstates_serial(key, hi, ho);
        }
        uint32_t t1[8], t2[8];
        {                                                // T1 = HMAC(PRK, 0x01)  (HKDF.py:56-60)
            uint32_t w[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) w[k] = 0u;
            w[0] = 0x01800000u;
            w[15] = (64u + 1u) * 8u;
#pragma unroll
            for (int k = 0; k < 8; ++k) inner[k] = hi[k];
            sha256_compress_fenced(inner, w);
            hmac_outer_fenced(t1, inner, ho);
        }
        if (NK == 8) {                                   // T2 = HMAC(PRK, T1 || 0x02)
            uint32_t w[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) w[k] = k < 8 ? t1[k] : 0u;
            w[8] = 0x02800000u;
            w[15] = (64u + 33u) * 8u;
#pragma unroll
            for (int k = 0; k < 8; ++k) inner[k] = hi[k];
            sha256_compress_fenced(inner, w);
            hmac_outer_fenced(t2, inner, ho);
        }
        // key = T1 || T2 (big-endian words): sk = key[:HALF], ek = key[HALF:]  (Token.py:61-70)
        uint32_t skw[16], ekw[NK];
#pragma unroll
        for (int k = 0; k < 16; ++k) skw[k] = k < (NK == 8 ? 8 : 4) ? t1[k] : 0u;
#pragma unroll
        for (int k = 0; k < NK; ++k) ekw[k] = bswap(NK == 8 ? t2[k] : t1[4 + k]);
        key_record<NK>(sb, ekw, skw, stage[wave], lane, kbase, a.n, rec_out);
    }
}

}  // namespace

hipError_t launch_hkdf(const HkdfArgs &a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    const uint32_t threads = 256;
    const auto aligned4 = [](const uint8_t *p, uint64_t stride) { return (((uintptr_t)p | stride) & 3u) == 0; };
    const bool fast = a.context_len == 0 && a.ikm_len % 4u == 0 && a.ikm_len <= 52u && aligned4(a.ikm, a.ikm_stride) &&
                      (a.salt == nullptr || (a.salt_len % 4u == 0 && a.salt_len <= 64u && aligned4(a.salt, a.salt_stride)));
#ifdef RNSTOK_NO_FAST_HKDF
    const bool use_fast = false && fast;
#else
    const bool use_fast = fast;
#endif
    // a shared salt row: 1024 x 256 lanes (4 waves per SIMD on 256 CUs), each
    // computing the salt's midstates once for its n / 262144 keys
#ifdef RNSTOK_NO_SHARED_SALT
    const bool shared = false;
#else
    const bool shared = a.salt != nullptr && a.salt_stride == 0 && a.n > 1;
#endif
    const uint64_t blocks = ((uint64_t)a.n + threads - 1) / threads;
    const dim3 grid((unsigned)(shared && blocks > 1024u ? 1024u : blocks));
    if (use_fast && shared)
        hipLaunchKernelGGL((k_hkdf<true, true>), grid, dim3(threads), 0, s, a);
    else if (use_fast)
        hipLaunchKernelGGL((k_hkdf<true, false>), grid, dim3(threads), 0, s, a);
    else if (shared)
        hipLaunchKernelGGL((k_hkdf<false, true>), grid, dim3(threads), 0, s, a);
    else
        hipLaunchKernelGGL((k_hkdf<false, false>), grid, dim3(threads), 0, s, a);
    return hipGetLastError();
}

#ifndef RNSTOK_FUSED_BLOCKS_PER_CU
#define RNSTOK_FUSED_BLOCKS_PER_CU 3      // 48 KiB of staging and 132 VGPRs: 3 workgroups of 4 waves per CU
#endif
hipError_t launch_hkdf_key_setup(const HkdfArgs &a, const uint8_t *sbox, uint32_t *rec, int n_cu, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
#ifdef RNSTOK_NO_FUSED_HKDF          // A/B: the two-launch path
    return hipErrorNotSupported;
#endif
    const auto aligned4 = [](const uint8_t *p, uint64_t stride) { return (((uintptr_t)p | stride) & 3u) == 0; };
    const bool fast = a.context_len == 0 && a.ikm_len % 4u == 0 && a.ikm_len <= 52u && aligned4(a.ikm, a.ikm_stride) &&
                      (a.salt == nullptr || (a.salt_len % 4u == 0 && a.salt_len <= 64u && aligned4(a.salt, a.salt_stride)));
    if (!fast || (a.length != 64u && a.length != 32u)) return hipErrorNotSupported;
    const bool shared = a.salt != nullptr && a.salt_stride == 0 && a.n > 1;
    uint64_t blocks = ((uint64_t)a.n + 255u) / 256u;
    if (shared && blocks > (uint64_t)RNSTOK_FUSED_BLOCKS_PER_CU * (uint64_t)n_cu)
        blocks = (uint64_t)RNSTOK_FUSED_BLOCKS_PER_CU * (uint64_t)n_cu;
    const dim3 grid((unsigned)blocks);
    if (a.length == 64u) {
        if (shared)
            hipLaunchKernelGGL((k_hkdf_key_setup<true, 8>), grid, dim3(256), 0, s, a, sbox, rec);
        else
            hipLaunchKernelGGL((k_hkdf_key_setup<false, 8>), grid, dim3(256), 0, s, a, sbox, rec);
    } else {
        if (shared)
            hipLaunchKernelGGL((k_hkdf_key_setup<true, 4>), grid, dim3(256), 0, s, a, sbox, rec);
        else
            hipLaunchKernelGGL((k_hkdf_key_setup<false, 4>), grid, dim3(256), 0, s, a, sbox, rec);
    }
    return hipGetLastError();
}

}  // namespace rnstok
