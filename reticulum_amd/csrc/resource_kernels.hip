// resource_kernels.hip — Resource hashmap (RNS/Resource.py:426-468, 505-506).
//
// A Resource is sent as one large token (Link.encrypt of random_hash(4) ||
// data, Resource.py:399-422) cut into SDU-sized parts (464 B for the default
// MTU, Resource.SDU = Packet.MDU).  Each part is advertised by its map hash
//     map_hash_j = SHA-256(part_j || random_hash)[:4]        (get_map_hash, :505-506)
// and the sender re-rolls random_hash whenever a map hash repeats one of the
// previous COLLISION_GUARD_SIZE (= 2*WINDOW_MAX + HASHMAP_MAX_LEN = 224) map
// hashes (:446-462).  The receiver recomputes the same hash for every part it
// gets (receive_part, :865-866).
//
// k_map_hashes: one lane per part.  The part's full 64-byte blocks are read
// with 16-byte loads (any alignment) and compressed; the last partial block,
// the random hash and the SHA padding are assembled from byte loads.  A part
// of 464 B is 8 compressions.  Parts of many resources can share a launch:
// part j belongs to resource part_res[j] and uses that resource's salt.
// k_map_collisions: for every part, compare its map hash with the previous
// `guard` parts of the same resource (parts of a resource are contiguous and
// in order) and record the first colliding index per resource (atomic min),
// which is where the reference's loop breaks out to re-roll.
#include "token_device.h"
#include "token_launch.h"

namespace rnstok {

namespace {

__device__ const uint32_t SHA_IV0[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                        0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

__device__ __forceinline__ uint32_t byte2(const uint8_t *a, uint32_t alen, const uint8_t *b, uint32_t blen,
                                          uint32_t q) {
    if (q < alen) return a[q];
    q -= alen;
    if (q < blen) return b[q];
    return q == blen ? 0x80u : 0u;
}

__global__ __launch_bounds__(256) void k_map_hashes(MapArgs m) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m.n_parts) return;
    const uint8_t *P = m.data + (m.part_off ? m.part_off[j] : (uint64_t)j * m.sdu);
    const uint32_t len = m.part_len ? m.part_len[j] : (uint32_t)min((uint64_t)m.sdu, m.size - (uint64_t)j * m.sdu);
    const uint32_t r = m.part_res ? m.part_res[j] : 0u;
    const uint8_t *S = m.salts + (uint64_t)r * m.salt_len;
    uint32_t h[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) h[k] = SHA_IV0[k];
    const uint32_t full = len >> 6;
    for (uint32_t b = 0; b < full; ++b) {
        const uint8_t *B = P + 64ull * b;
        uint32_t w[16];
        sha_units(w, ld16(B), ld16(B + 16), ld16(B + 32), ld16(B + 48));
        sha256_compress(h, w);
    }
    // tail: rem bytes of the part || salt || 0x80 || zeros || bit length (1 or 2 blocks)
    const uint32_t rem = len - 64u * full;
    const uint8_t *T = P + 64ull * full;
    const uint64_t bits = ((uint64_t)len + m.salt_len) * 8u;
    const uint32_t tb = (rem + m.salt_len + 8u) / 64u + 1u;
    for (uint32_t b = 0; b < tb; ++b) {
        uint32_t w[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t q = 64u * b + 4u * k;
            w[k] = (byte2(T, rem, S, m.salt_len, q) << 24) | (byte2(T, rem, S, m.salt_len, q + 1) << 16) |
                   (byte2(T, rem, S, m.salt_len, q + 2) << 8) | byte2(T, rem, S, m.salt_len, q + 3);
        }
        if (b + 1 == tb) {
            w[14] = (uint32_t)(bits >> 32);
            w[15] = (uint32_t)bits;
        }
        sha256_compress(h, w);
    }
    // digest[:4] = big-endian first state word (MAPHASH_LEN = 4)
    const uint32_t d = bswap(h[0]);
    __builtin_memcpy(m.out + 4ull * j, &d, 4);
}

__global__ __launch_bounds__(256) void k_map_collisions(MapArgs m) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m.n_parts) return;
    const uint32_t r = m.part_res ? m.part_res[j] : 0u;
    uint32_t mine, other;
    __builtin_memcpy(&mine, m.out + 4ull * j, 4);
    const uint32_t lo = j > m.guard ? j - m.guard : 0u;
    for (uint32_t k = lo; k < j; ++k) {
        if (m.part_res && m.part_res[k] != r) continue;
        __builtin_memcpy(&other, m.out + 4ull * k, 4);
        if (other == mine) {
            atomicMin(m.first_collision + r, j);
            break;
        }
    }
}

}  // namespace

// The same comparison with the workgroup's window of map hashes (its 256
// parts and the `guard` parts before them) staged in LDS once, instead of
// every lane reading its `guard` predecessors from memory (0.12 ms of
// global reads per 2^20 parts at guard 224).
constexpr uint32_t COLL_TILE = 256, COLL_LDS_GUARD_MAX = 4096;
__global__ __launch_bounds__(COLL_TILE) void k_map_collisions_lds(MapArgs m) {
    extern __shared__ uint32_t win[];                 // [span] hashes, then [span] resource ids
    const uint32_t j0 = blockIdx.x * COLL_TILE, lo = j0 > m.guard ? j0 - m.guard : 0u;
    const uint32_t hi = j0 + COLL_TILE < m.n_parts ? j0 + COLL_TILE : m.n_parts, span = hi - lo;
    uint32_t *res = win + m.guard + COLL_TILE;
    for (uint32_t k = threadIdx.x; k < span; k += COLL_TILE) {
        uint32_t v;
        __builtin_memcpy(&v, m.out + 4ull * (lo + k), 4);
        win[k] = v;
        res[k] = m.part_res ? m.part_res[lo + k] : 0u;
    }
    __syncthreads();
    const uint32_t j = j0 + threadIdx.x;
    if (j >= m.n_parts) return;
    const uint32_t mine = win[j - lo], r = res[j - lo];
    const uint32_t from = j > m.guard ? j - m.guard : 0u;
    if (res[0] == res[span - 1]) {               // the window is one resource (parts are contiguous)
        for (uint32_t k = from; k < j; ++k) {
            if (win[k - lo] == mine) {
                atomicMin(m.first_collision + r, j);
                break;
            }
        }
        return;
    }
    for (uint32_t k = from; k < j; ++k) {
        if (res[k - lo] == r && win[k - lo] == mine) {
            atomicMin(m.first_collision + r, j);
            break;
        }
    }
}

hipError_t launch_map_hashes(const MapArgs &m, hipStream_t s) {
    if (m.n_parts == 0) return hipSuccess;
    const uint32_t threads = 256, grid = (m.n_parts + threads - 1) / threads;
    hipLaunchKernelGGL(k_map_hashes, dim3(grid), dim3(threads), 0, s, m);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !m.first_collision) return e;
    e = hipMemsetAsync(m.first_collision, 0xff, 4ull * m.n_res, s);      // "no collision" = 0xffffffff
    if (e != hipSuccess) return e;
    if (m.guard == 0) return hipSuccess;
    if (m.guard <= COLL_LDS_GUARD_MAX)
        hipLaunchKernelGGL(k_map_collisions_lds, dim3((m.n_parts + COLL_TILE - 1) / COLL_TILE), dim3(COLL_TILE),
                           8u * (m.guard + COLL_TILE), s, m);
    else
        hipLaunchKernelGGL(k_map_collisions, dim3(grid), dim3(threads), 0, s, m);
    return hipGetLastError();
}

}  // namespace rnstok
