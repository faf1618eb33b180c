// copy_kernels.hip — device-to-host copies as GPU stores into pinned host
// memory (the host-origin path of SURVEY §8(d): packets start and end in
// socket buffers, TCPInterface.py:392-401 -> Link.py:1161-1182).
//
// Measured on MI355X (tools/pcie_probe.hip, profiles/r03n_pcie_probe.json):
// the runtime's copy engine moves device->host at 30 GB/s and host->device
// at 57 GB/s, and the two directions at once share 57 GB/s; a kernel whose
// waves store 16 B per lane (1 KiB contiguous per wave instruction) into the
// mapped host buffer reaches 54 GB/s, and beside a copy-engine H2D the link
// carries 87 GB/s in total.  So H2D stays on hipMemcpyAsync and D2H of
// pinned destinations runs here.
#include <algorithm>

#include "token_launch.h"

namespace rnstok {

namespace {

typedef unsigned int u32x4c __attribute__((ext_vector_type(4)));

// dst + head is 16-B aligned; the body is `body` aligned 16-B stores, the
// head and tail bytes are stored one by one by the first 32 threads.  With
// `dev_bytes` the byte count is min(bytes, *dev_bytes), read on the device
// (a size the host does not know, e.g. the end offset of an HDLC stream),
// read as a signed int64 so that a negative count copies nothing.
__global__ __launch_bounds__(256) void k_store_host(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                    uint64_t bytes, uint32_t head, const uint64_t *dev_bytes) {
    if (dev_bytes) {
        // a signed count (torch int64): zero or negative copies nothing
        const int64_t d = (int64_t)*dev_bytes;
        bytes = d <= 0 ? 0u : ((uint64_t)d < bytes ? (uint64_t)d : bytes);
        head = (uint32_t)(head < bytes ? head : bytes);
    }
    const uint64_t body = (bytes - head) >> 4;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint8_t *s = src + head;
    u32x4c *d = (u32x4c *)(dst + head);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < body; i += stride) {
        u32x4c v;
        __builtin_memcpy(&v, s + 16 * i, 16);      // any source alignment: global_load_dwordx4
        d[i] = v;
    }
    if (blockIdx.x == 0 && threadIdx.x < 32u) {
        const uint32_t t = threadIdx.x & 15u;
        const uint64_t at = threadIdx.x < 16u ? t : head + 16 * body + t;
        if ((threadIdx.x < 16u ? t < head : at < bytes)) dst[at] = src[at];
    }
}

}  // namespace

hipError_t launch_store_host(uint8_t *dst_dev, const uint8_t *src, uint64_t bytes, hipStream_t s,
                             const uint64_t *dev_bytes) {
    if (!bytes) return hipSuccess;
    const uint32_t head = (uint32_t)std::min<uint64_t>((16u - ((uintptr_t)dst_dev & 15u)) & 15u, bytes);
    const uint64_t body = (bytes - head) >> 4;
    const uint64_t blocks = std::max<uint64_t>(1, std::min<uint64_t>((body + 255) / 256, 2048));
    hipLaunchKernelGGL(k_store_host, dim3((unsigned)blocks), dim3(256), 0, s, src, dst_dev, bytes, head, dev_bytes);
    return hipGetLastError();
}

}  // namespace rnstok
