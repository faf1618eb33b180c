"""Generate tools/issue_model_probe.hip: what sets the VALU issue cost on gfx950.

VERDICT r02 asked what makes a full-rate VALU op cost 2.40 (4-byte VOP2) /
2.59 (8-byte) SIMD-cycles per wave64 instruction at 4 waves/SIMD in
tools/cost_probe.hip, against the guide's 2.0.  Hypotheses tested here, each
as a kernel of its own so one rocprofv3 --pmc pass attributes counters
(SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU2, SQ_INSTS_LDS, SQ_IFETCH, ...) per case:

  W  waves per SIMD (1, 2, 3, 4, 8): is the cost a shortage of ready waves?
  E  encoding: the same v_xor_b32 as 4-byte VOP2 and as 8-byte VOP3 (_e64),
     a literal operand, v_bitop3, half-rate forms, an SGPR operand
  C  independent chains per wave (1 ... 16): dependency latency?
  B  VGPR banks (register index mod 4) of the chains and of the shared source
  M  mixes: full-rate ops interleaved with / clustered apart from half-rate
     ones; ds_read_b32 lookups beside full-rate and beside half-rate ops
     (does a lookup take a VALU issue slot?)
  L  loop body length (64 vs 512 instructions per iteration): branch and
     instruction-fetch cost per instruction

All chains live in explicitly named VGPRs (v20..v51, clobbered) so the
register banks are known.  Wave 0 of every workgroup stamps s_memtime /
s_memrealtime around the loop; the host prints SIMD-cycles per
wave-iteration at the in-kernel clock.

  python3 tools/gen_issue_model_probe.py   # writes tools/issue_model_probe.hip
  hipcc --offload-arch=gfx950 -O3 -o build_exp/issue_model_probe tools/issue_model_probe.hip
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))

CLOB = ", ".join('"v%d"' % r for r in range(20, 56))

# Each case: name, threads per WG, WGs per CU, body text (one iteration),
# VALU per wave-iteration, LDS per wave-iteration, doc.
CASES = []


def rep(f, n):
    return "".join(f(i) for i in range(n))


def chain_body(op, nchains=8, n=64, dst=None, src="v52", src2="v53"):
    """n instructions of `op` cycling over nchains destination registers."""
    dst = dst or [20 + i for i in range(nchains)]
    out = []
    for i in range(n):
        d = "v%d" % dst[i % len(dst)]
        out.append(op.format(d=d, s=src, t=src2))
    return out


XOR32 = "v_xor_b32 {d}, {s}, {d}"
XOR64 = "v_xor_b32_e64 {d}, {s}, {d}"
ADDLIT = "v_add_u32 {d}, 0x428a2f98, {d}"
ADD32 = "v_add_u32 {d}, {s}, {d}"
BITOP3 = "v_bitop3_b32 {d}, {d}, {s}, {t} bitop3:0x96"
PERM = "v_perm_b32 {d}, {d}, {s}, {t}"
ALIGN = "v_alignbit_b32 {d}, {d}, {d}, 7"
ADD3 = "v_add3_u32 {d}, {d}, {s}, {t}"
XORS = "v_xor_b32 {d}, s60, {d}"
LSHR = "v_lshrrev_b32 {d}, 9, {d}"


def add(name, body, valu, lds=0, threads=1024, wgs=1, doc="", body_b=None):
    """body_b: waves ranked 2-3 on their hardware SIMD run body_b instead of body
    (role split inside every SIMD: 2 waves of each kind)."""
    CASES.append(dict(name=name, body=body, valu=valu, lds=lds, threads=threads, wgs=wgs, doc=doc, body_b=body_b))


# W: waves per SIMD
for op, tag in ((XOR32, "xor32"), (BITOP3, "bitop3"), (PERM, "perm")):
    for thr, wgs, w in ((256, 1, 1), (512, 1, 2), (768, 1, 3), (1024, 1, 4), (1024, 2, 8)):
        add("W_%s_w%d" % (tag, w), chain_body(op), 64, threads=thr, wgs=wgs, doc="%s, %d waves/SIMD" % (tag, w))

# E: encodings at 4 waves/SIMD
for op, tag in ((XOR32, "xor_vop2_4B"), (XOR64, "xor_vop3_8B"), (ADD32, "add_vop2_4B"), (ADDLIT, "add_literal_8B"),
                (BITOP3, "bitop3_8B"), (LSHR, "lshr_imm_4B"), (PERM, "perm_8B"), (ALIGN, "alignbit_8B"),
                (ADD3, "add3_8B"), (XORS, "xor_sgpr_4B")):
    add("E_" + tag, chain_body(op), 64, doc=tag)

# C: chains per wave
for nc in (1, 2, 4, 8, 16):
    add("C_xor32_chains%d" % nc, chain_body(XOR32, nchains=nc), 64, doc="%d chains" % nc)
    add("C_bitop3_chains%d" % nc, chain_body(BITOP3, nchains=nc), 64, doc="%d chains" % nc)

# B: banks.  chains on v20..v27 (banks 0,1,2,3,0,1,2,3) is the default;
# all chains in bank 0 (v20, v24, ... v48) with the source in bank 0 or 1.
bank0 = [20 + 4 * i for i in range(8)]
add("B_xor32_dst_bank0_src_bank0", chain_body(XOR32, dst=bank0, src="v52"), 64, doc="dst banks all 0, src bank 0")
add("B_xor32_dst_bank0_src_bank1", chain_body(XOR32, dst=bank0, src="v53"), 64, doc="dst banks all 0, src bank 1")
add("B_bitop3_all_bank0", chain_body(BITOP3, dst=bank0, src="v52", src2="v44"), 64, doc="d,s,t all bank 0")
add("B_bitop3_banks_012", chain_body(BITOP3, dst=bank0, src="v53", src2="v54"), 64, doc="d bank 0, s 1, t 2")

# M: mixes (4 waves/SIMD)
x = chain_body(XOR32, n=32)
p = chain_body(PERM, n=32, dst=[28 + i for i in range(8)])
add("M_xor32_perm_alternate", [v for pair in zip(x, p) for v in pair], 64, doc="32 xor + 32 perm, alternating")
add("M_xor32_perm_clustered", x + p, 64, doc="32 xor then 32 perm")
x3 = chain_body(XOR32, n=48)
p3 = chain_body(PERM, n=16, dst=[28 + i for i in range(8)])
add("M_xor48_perm16_alternate", [v for i in range(16) for v in (x3[3 * i], x3[3 * i + 1], x3[3 * i + 2], p3[i])], 64,
    doc="48 xor + 16 perm, 3:1")
xs = chain_body(XORS, n=32, dst=[28 + i for i in range(8)])
add("M_xor32_xorsgpr_alternate", [v for pair in zip(x, xs) for v in pair], 64, doc="32 xor v,v + 32 xor s,v")


def with_lds(valu_body, nlds):
    """interleave nlds ds_read_b32 (conflict-free: v54 = 4*lane + row) into valu_body,
    results into v40..v47 (not read by the VALU chains), one wait at the end."""
    out = []
    step = len(valu_body) // nlds if nlds else 0
    k = 0
    for i, ins in enumerate(valu_body):
        if nlds and i % step == 0 and k < nlds:
            if k and k % 8 == 0:
                out.append("s_waitcnt lgkmcnt(8)")
            out.append("ds_read_b32 v%d, v54 offset:%d" % (40 + (k % 8), 256 * (k % 16)))
            k += 1
        out.append(ins)
    if nlds:
        out.append("s_waitcnt lgkmcnt(0)")
    return out


for n in (0, 8, 16, 32):
    add("M_xor32x64_lds%d" % n, with_lds(chain_body(XOR32), n), 64, n, doc="64 xor + %d ds_read_b32" % n)
    add("M_perm64_lds%d" % n, with_lds(chain_body(PERM), n), 64, n, doc="64 perm + %d ds_read_b32" % n)
    add("M_bitop3x64_lds%d" % n, with_lds(chain_body(BITOP3), n), 64, n, doc="64 bitop3 + %d ds_read_b32" % n)

# K: run length of full-rate vs half-rate ops (512-instruction body: 256 xor +
# 256 perm in runs of k, alternating)
xs512 = chain_body(XOR32, n=256)
ps512 = chain_body(PERM, n=256, dst=[28 + i for i in range(8)])
for k in (1, 4, 16, 64, 256):
    body = []
    for r in range(0, 256, k):
        body += xs512[r:r + k] + ps512[r:r + k]
    add("K_xor_perm_runs%d" % k, body, 512, doc="256 xor + 256 perm in alternating runs of %d" % k)

# P: lookups beside full-rate ops in a 512-instruction body (no loop overhead)
for every in (4, 8, 16):
    add("P_xor512_lds_every%d" % every, with_lds(chain_body(XOR32, n=512), 512 // every), 512, 512 // every,
        doc="512 xor + one ds_read_b32 per %d" % every)
    add("P_perm512_lds_every%d" % every, with_lds(chain_body(PERM, n=512), 512 // every), 512, 512 // every,
        doc="512 perm + one ds_read_b32 per %d" % every)

# S: roles split inside every SIMD (ranks 0-1 one stream, ranks 2-3 the other)
add("S_split_xor_vs_perm", chain_body(XOR32, n=512), 512, doc="2 waves xor | 2 waves perm per SIMD",
    body_b=chain_body(PERM, n=512, dst=[28 + i for i in range(8)]))
add("S_split_xor_vs_xor", chain_body(XOR32, n=512), 512, doc="control: 4 waves xor, split code path",
    body_b=chain_body(XOR32, n=512, dst=[28 + i for i in range(8)]))
add("S_split_xor_vs_lds", chain_body(XOR32, n=512), 512, doc="2 waves xor | 2 waves 64 ds_read + 448 xor",
    body_b=with_lds(chain_body(XOR32, n=448, dst=[28 + i for i in range(8)]), 64))

# X: the token kernel's round mixes.  One AES T-table round (16 ds_read_b32,
# 12 v_perm byte addresses + 4 and_or, 8 xor3 of which 4 take the round key
# from an SGPR) and one SHA-256 round (6 v_alignbit, 2 v_add3, 4 bitop3, 3
# v_add), as k_encrypt interleaves them; an "eligible" AES form builds the 12
# addresses with a shift + and_or each (all dual-issuable) and keeps the key in
# VGPRs.  Mixed: every wave runs AES+SHA rounds; split: two waves per SIMD run
# only AES rounds and two only SHA rounds (the same total work per SIMD).
def aes_round(elig, vkey=None):
    vkey = elig if vkey is None else vkey
    out = []
    for k in range(16):
        if k % 4 == 1:
            out.append("v_bitop3_b32 v%d, v%d, v53, v52 bitop3:0xea" % (28 + k % 8, 20 + k // 4))
        elif elig:
            out.append("v_lshrrev_b32 v%d, %d, v%d" % (28 + k % 8, 8 * (k % 4), 20 + k // 4))
            out.append("v_bitop3_b32 v%d, v%d, v53, v52 bitop3:0xea" % (28 + k % 8, 28 + k % 8))
        else:
            out.append("v_perm_b32 v%d, v%d, v52, s60" % (28 + k % 8, 20 + k // 4))
        out.append("ds_read_b32 v%d, v54 offset:%d" % (40 + k % 8, 256 * k))
        if k % 8 == 7:
            out.append("s_waitcnt lgkmcnt(4)")
    out.append("s_waitcnt lgkmcnt(0)")
    for j in range(4):
        out.append("v_bitop3_b32 v%d, v%d, v%d, v%d bitop3:0x96" % (36 + j, 40 + 2 * j, 41 + 2 * j, 29 + 2 * j))
        if vkey:
            out.append("v_bitop3_b32 v%d, v%d, v%d, v%d bitop3:0x96" % (20 + j, 36 + j, 42 + (2 * j) % 8, 55))
        else:
            out.append("v_bitop3_b32 v%d, v%d, v%d, s60 bitop3:0x96" % (20 + j, 36 + j, 42 + (2 * j) % 8))
    return out


def sha_round():
    return ["v_alignbit_b32 v44, v24, v24, 6", "v_alignbit_b32 v45, v24, v24, 11", "v_alignbit_b32 v46, v24, v24, 25",
            "v_bitop3_b32 v47, v44, v45, v46 bitop3:0x96", "v_bitop3_b32 v49, v24, v25, v26 bitop3:0xca",
            "v_add3_u32 v50, v27, v53, v48", "v_add3_u32 v50, v50, v47, v49",
            "v_alignbit_b32 v44, v21, v21, 2", "v_alignbit_b32 v45, v21, v21, 13", "v_alignbit_b32 v46, v21, v21, 22",
            "v_bitop3_b32 v47, v44, v45, v46 bitop3:0x96", "v_bitop3_b32 v49, v21, v22, v23 bitop3:0xe8",
            "v_add_u32 v51, v47, v49", "v_add_u32 v25, v25, v50", "v_add_u32 v24, v50, v51"]


for elig in (False, True):
    tag = "elig" if elig else "perm"
    a, h = aes_round(elig), sha_round()
    add("X_mixed_%s" % tag, (a + h) * 8, len([i for i in (a + h) * 8 if i.startswith("v_")]),
        doc="every wave: 8 x (AES round, %s form + SHA round)" % tag)
    add("X_split_%s" % tag, a * 16, len([i for i in (a + h) * 8 if i.startswith("v_")]),
        doc="2 waves 16 AES rounds (%s form) | 2 waves 16 SHA rounds" % tag, body_b=h * 16)
    add("X_aesonly_%s" % tag, a * 16, len([i for i in a * 16 if i.startswith("v_")]),
        doc="every wave: 16 AES rounds (%s form)" % tag)
for elig, vkey, tag in ((True, False, "elig_skey"), (False, True, "perm_vkey")):
    a, h = aes_round(elig, vkey), sha_round()
    add("X_mixed_%s" % tag, (a + h) * 8, len([i for i in (a + h) * 8 if i.startswith("v_")]),
        doc="every wave: 8 x (AES round, %s + SHA round)" % tag)
add("X_shaonly", sha_round() * 16, 15 * 16, doc="every wave: 16 SHA rounds")

# L: body length
add("L_xor32_body512", chain_body(XOR32, n=512), 512, doc="512 xor per iteration")
add("L_perm_body512", chain_body(PERM, n=512), 512, doc="512 perm per iteration")


HEAD = r'''// issue_model_probe.hip — GENERATED by tools/gen_issue_model_probe.py (do not edit).
// What sets the VALU issue cost on gfx950; see the generator's docstring.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

struct Stamp { unsigned long long t0, t1, r0, r1; };

__device__ __forceinline__ unsigned long long memtime() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
__device__ __forceinline__ unsigned long long memrealtime() {
    unsigned long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

// rank of this wave among the waves of its hardware SIMD (HW_ID), from an
// LDS counter at the top of the 64 KiB the kernel always has
__device__ __forceinline__ uint32_t simd_rank() {
    typedef __attribute__((address_space(3))) uint32_t l32w;
    l32w *cnt = (l32w *)(uintptr_t)(65536 - 64);
    if (threadIdx.x < 4) cnt[threadIdx.x] = 0;
    __syncthreads();
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    const uint32_t simd = (hw >> 4) & 3u;
    uint32_t rank = 0;
    if ((threadIdx.x & 63u) == 0) rank = __hip_atomic_fetch_add(&cnt[simd], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    rank = __builtin_amdgcn_readfirstlane(rank);
    __syncthreads();
    return rank;
}

#define INIT_REGS()                                                                        \
    asm volatile(                                                                          \
        "v_mov_b32 v20, %0\n v_add_u32 v21, 1, v20\n v_add_u32 v22, 2, v20\n v_add_u32 v23, 3, v20\n" \
        "v_add_u32 v24, 4, v20\n v_add_u32 v25, 5, v20\n v_add_u32 v26, 6, v20\n v_add_u32 v27, 7, v20\n" \
        "v_add_u32 v28, 8, v20\n v_add_u32 v29, 9, v20\n v_add_u32 v30, 10, v20\n v_add_u32 v31, 11, v20\n" \
        "v_add_u32 v32, 12, v20\n v_add_u32 v33, 13, v20\n v_add_u32 v34, 14, v20\n v_add_u32 v35, 15, v20\n" \
        "v_add_u32 v36, 16, v20\n v_add_u32 v37, 17, v20\n v_add_u32 v38, 18, v20\n v_add_u32 v39, 19, v20\n" \
        "v_add_u32 v44, 20, v20\n v_add_u32 v48, 21, v20\n" \
        "v_mov_b32 v52, %1\n v_mov_b32 v53, %2\n v_mov_b32 v54, %3\n s_mov_b32 s60, %4\n"  \
        :: "v"(threadIdx.x ^ seed), "v"(seed * 3u), "v"(seed * 5u + threadIdx.x),          \
           "v"(4u * (threadIdx.x & 31u)), "s"(seed * 7u) : CLOBBERS, "s60")

#define STAMP_BEGIN()                                                                      \
    unsigned long long t0 = 0, r0 = 0;                                                     \
    __syncthreads();                                                                       \
    if (threadIdx.x == 0) { t0 = memtime(); r0 = memrealtime(); }

#define STAMP_END()                                                                        \
    __syncthreads();                                                                       \
    if (threadIdx.x == 0) {                                                                \
        unsigned long long t1 = memtime(), r1 = memrealtime();                             \
        st[blockIdx.x].t0 = t0; st[blockIdx.x].t1 = t1; st[blockIdx.x].r0 = r0; st[blockIdx.x].r1 = r1; \
    }                                                                                      \
    uint32_t acc;                                                                          \
    asm volatile("v_xor_b32 %0, v20, v21\n v_bitop3_b32 %0, %0, v28, v40 bitop3:0x96" : "=v"(acc) :: CLOBBERS); \
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
'''


def emit():
    lines = [HEAD.replace("CLOBBERS", CLOB)]
    for c in CASES:
        bounds = "%d, %d" % (c["threads"], max(1, c["threads"] // 256 * c["wgs"]))
        asm = "\\n".join(c["body"])
        lines.append('// %s: %s' % (c["name"], c["doc"]))
        lines.append('__global__ __launch_bounds__(%s) void k_%s(uint32_t *out, Stamp *st, uint32_t seed, int iters) {'
                     % (bounds, c["name"]))
        lines.append("    INIT_REGS();".replace("CLOBBERS", CLOB))
        lines.append("    STAMP_BEGIN();")
        if c["body_b"] is None:
            lines.append("    for (int i = 0; i < iters; ++i) {")
            lines.append('        asm volatile("%s" ::: %s, "s60", "memory");' % (asm, CLOB))
            lines.append("    }")
        else:
            asm_b = "\\n".join(c["body_b"])
            lines.append("    if (simd_rank() < 2u) {")
            lines.append("        for (int i = 0; i < iters; ++i) {")
            lines.append('            asm volatile("%s" ::: %s, "s60", "memory");' % (asm, CLOB))
            lines.append("        }")
            lines.append("    } else {")
            lines.append("        for (int i = 0; i < iters; ++i) {")
            lines.append('            asm volatile("%s" ::: %s, "s60", "memory");' % (asm_b, CLOB))
            lines.append("        }")
            lines.append("    }")
        lines.append("    STAMP_END();".replace("CLOBBERS", CLOB))
        lines.append("}")
        lines.append("")
    lines.append("typedef void (*kfn)(uint32_t *, Stamp *, uint32_t, int);")
    lines.append("struct Case { const char *name; kfn k; int threads, wgs, valu, lds; const char *doc; };")
    lines.append("static const Case CASES[] = {")
    for c in CASES:
        lines.append('    {"%s", k_%s, %d, %d, %d, %d, "%s"},' % (c["name"], c["name"], c["threads"], c["wgs"],
                                                                  c["valu"], c["lds"], c["doc"]))
    lines.append("};")
    lines.append(TAIL)
    with open(os.path.join(HERE, "issue_model_probe.hip"), "w") as f:
        f.write("\n".join(lines))


TAIL = r'''
int main(int argc, char **argv) {
    const char *filter = argc > 1 ? argv[1] : "";
    const int iters = argc > 2 ? atoi(argv[2]) : 2000;
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int ncu = p.multiProcessorCount;
    uint32_t *d_out;
    Stamp *d_st;
    CHECK(hipMalloc(&d_out, 4ull * ncu * 2 * 1024));
    CHECK(hipMalloc(&d_st, sizeof(Stamp) * ncu * 2));
    Stamp *h = (Stamp *)malloc(sizeof(Stamp) * ncu * 2);
    printf("%-30s %5s %5s %4s %8s %6s %10s %8s %9s  %s\n", "case", "w/SI", "VALU", "LDS", "ms", "GHz",
           "cyc/it/SI", "cyc/VALU", "slots/it", "doc");
    const int n = sizeof(CASES) / sizeof(CASES[0]);
    for (int c = 0; c < n; ++c) {
        const Case &cs = CASES[c];
        if (filter[0] && !strstr(cs.name, filter)) continue;
        const int lds = cs.wgs == 1 ? 131072 : 65536;   // pins wgs workgroups per CU
        CHECK(hipFuncSetAttribute((const void *)cs.k, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        const int grid = ncu * cs.wgs;
        hipLaunchKernelGGL(cs.k, dim3(grid), dim3(cs.threads), lds, 0, d_out, d_st, 1u, iters);
        CHECK(hipDeviceSynchronize());
        float best = 1e30f;
        double ghz = 0, cyc = 0;
        hipEvent_t e0, e1;
        CHECK(hipEventCreate(&e0));
        CHECK(hipEventCreate(&e1));
        for (int r = 0; r < 5; ++r) {
            CHECK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(cs.k, dim3(grid), dim3(cs.threads), lds, 0, d_out, d_st, 2u + r, iters);
            CHECK(hipEventRecord(e1, 0));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) {
                best = ms;
                CHECK(hipMemcpy(h, d_st, sizeof(Stamp) * grid, hipMemcpyDeviceToHost));
                double sum = 0, mx = 0;
                for (int b = 0; b < grid; ++b) {
                    const double d = (double)(h[b].t1 - h[b].t0);
                    sum += d / (double)(h[b].r1 - h[b].r0) * 0.1;
                    mx = d > mx ? d : mx;
                }
                ghz = sum / grid;
                cyc = mx;
            }
        }
        CHECK(hipEventDestroy(e0));
        CHECK(hipEventDestroy(e1));
        const double wps = cs.threads / 64.0 / 4.0 * cs.wgs;     // waves per SIMD
        const double per_it = cyc / (wps * iters);                // SIMD-cycles per wave-iteration
        printf("%-30s %5.0f %5d %4d %8.3f %6.2f %10.1f %8.2f %9.1f  %s\n", cs.name, wps, cs.valu, cs.lds, best, ghz,
               per_it, per_it / cs.valu, per_it / 4.0, cs.doc);
        fflush(stdout);
    }
    free(h);
    return 0;
}
'''

if __name__ == "__main__":
    emit()
    print("wrote", os.path.join(HERE, "issue_model_probe.hip"), len(CASES), "cases")
