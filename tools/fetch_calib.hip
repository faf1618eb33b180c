// fetch_calib.hip — calibrate rocprofv3 FETCH_SIZE on the token kernels' own
// access pattern (MI355X_MICROARCH.md §HBM: the x2 correction is measured for
// coalesced 16-B streams; "other access widths are uncalibrated").
//
// k_packets: like k_encrypt's plaintext reads — lane p reads packet p
// (500 B at a 500-B stride) as 16-B loads, 64 B per step, one step per
// "quad" (with a VALU delay between steps, as the AES chain has).
// k_stream: the coalesced control — consecutive lanes read consecutive 16 B.
// Both read the same 2^20 x 500 B = 524 288 000 bytes once; each writes 4 B
// per lane.  Run each under `rocprofv3 --pmc FETCH_SIZE` and compare.
//   hipcc --offload-arch=gfx950 -O3 -o tools/_bin/fetch_calib tools/fetch_calib.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4 ld16(const uint8_t *p) {
    u32x4 v;
    __builtin_memcpy(&v, p, 16);
    return v;
}

constexpr uint32_t N = 1u << 20, L = 500;

__global__ __launch_bounds__(1024) void k_packets(const uint8_t *pt, uint32_t *out, int spin) {
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < N; p += gridDim.x * blockDim.x) {
        const uint8_t *P = pt + (uint64_t)p * L;
        uint32_t acc = p;
        for (uint32_t q = 0; q < L / 64; ++q) {          // 7 full quads
            const u32x4 a = ld16(P + 64 * q), b = ld16(P + 64 * q + 16), c = ld16(P + 64 * q + 32),
                        d = ld16(P + 64 * q + 48);
            acc ^= a.x ^ b.y ^ c.z ^ d.w ^ a.w ^ b.x ^ c.y ^ d.z;
            for (int k = 0; k < spin; ++k) acc = acc * 2654435761u + 1u;   // the AES chain's pace
        }
        for (uint32_t k = 64 * (L / 64); k < L; ++k) acc ^= P[k];         // the tail, byte by byte
        out[p] = acc;
    }
}

// k_rows: like k_decrypt's token reads — lane p reads row p (560 B = 35 16-B
// units at a ROW-byte stride, first row at byte OFF), the IV first, then the
// units in groups of 8 (the paired quads), a VALU delay between groups.
// Known bytes: N x 560.  ROW 560 / OFF 0: packed c2 tokens; ROW 640 / OFF 112:
// each token's ciphertext on a 128-B line.
template <uint32_t ROW, uint32_t OFF>
__global__ __launch_bounds__(768) void k_rows(const uint8_t *tok, uint32_t *out, int spin) {
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < N; p += gridDim.x * blockDim.x) {
        const uint8_t *P = tok + OFF + (uint64_t)p * ROW;
        u32x4 acc = ld16(P);
        for (uint32_t g = 0; g < 34u; g += 8u) {
            u32x4 v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = g + 1u + k < 35u ? ld16(P + 16 * (g + 1u + k)) : acc;
#pragma unroll
            for (int k = 0; k < 8; ++k) acc ^= v[k];
            for (int k = 0; k < spin; ++k) acc.x = acc.x * 2654435761u + 1u;
        }
        out[p] = acc.x ^ acc.y ^ acc.z ^ acc.w;
    }
}

__global__ __launch_bounds__(256) void k_stream(const uint8_t *pt, uint32_t *out) {
    const uint64_t n16 = (uint64_t)N * L / 16;
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        const u32x4 a = ld16(pt + 16 * i);
        acc ^= a.x ^ a.y ^ a.z ^ a.w;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main(int argc, char **argv) {
    const char *which = argc > 1 ? argv[1] : "packets";
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int ncu = prop.multiProcessorCount;
    uint8_t *pt;
    uint32_t *out;
    CHECK(hipMalloc(&pt, (uint64_t)N * 640 + 256));
    CHECK(hipMalloc(&out, 4ull * N));
    CHECK(hipMemset(pt, 0x5a, (uint64_t)N * 640 + 256));
    for (int r = 0; r < 3; ++r) {
        if (strcmp(which, "stream") == 0)
            hipLaunchKernelGGL(k_stream, dim3(ncu * 8), dim3(256), 0, 0, pt, out);
        else if (strcmp(which, "rows560") == 0)
            hipLaunchKernelGGL((k_rows<560, 0>), dim3(ncu), dim3(768), 0, 0, pt, out, 400);
        else if (strcmp(which, "rows640") == 0)
            hipLaunchKernelGGL((k_rows<640, 112>), dim3(ncu), dim3(768), 0, 0, pt, out, 400);
        else
            hipLaunchKernelGGL(k_packets, dim3(ncu), dim3(1024), 0, 0, pt, out, 200);
        CHECK(hipDeviceSynchronize());
    }
    printf("%s: %llu bytes read per launch (algorithmic)\n", which,
           (unsigned long long)N * (strncmp(which, "rows", 4) == 0 ? 560u : L));
    return 0;
}
