// token_capi.hip — C-ABI of librnstok.so (declared in include/rnstok.h).
//
// Host-side runtime around the kernels: device contexts, key tables, argument
// validation, host staging for the PCIe-inclusive path.  No exceptions cross
// the boundary; errors are negative RT_E_* codes plus rt_last_error().
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rnstok.h"
#include "token_device.h"
#include "token_launch.h"

using namespace rnstok;

// A host-staging lane: a private stream, a device workspace and a pinned
// mirror of it.  The context keeps N_STAGERS of them, so host calls from
// several threads (e.g. one reader thread per interface) run concurrently
// instead of queueing on one lock; a call takes a free lane or waits for one.
struct Stager {
    std::mutex mu;
    hipStream_t stream = nullptr;
    uint8_t *d_work = nullptr;     // host-path workspace
    uint64_t work_cap = 0;
    // Pinned mirror of the workspace for token host calls up to STAGE_MAX
    // bytes: the caller's arrays are gathered here and cross PCIe as one copy
    // each way.  A pageable copy pays a driver staging round trip per array
    // (6 of them per encrypt), which dominates a one-packet Token.encrypt.
    uint8_t *h_stage = nullptr;
    uint8_t *h_stage_dev = nullptr;    // its device-side address (GPU stores, launch_store_host)
    uint64_t stage_cap = 0;
    bool stage_busy = false;       // a copy from h_stage may still be queued on `stream`
};
// 8 lanes (round 6): one Token call per packet from 16 threads, 44 600 ->
// 73 000 calls/s against 4 lanes (two runs each, profiles/r06_percall_lanes.txt;
// one thread unchanged at 19 000); streams beyond the box's four hardware
// queues still overlap the host-side waits of concurrent calls.  Pinned
// staging grows on demand, at most 8 MiB per lane.
#ifndef RNSTOK_N_STAGERS
#define RNSTOK_N_STAGERS 8
#endif
static constexpr int N_STAGERS = RNSTOK_N_STAGERS;

// Chunk counters for the token kernels' dynamic packet loop (ragged uniform
// batches): one 64-B slot per launch.  A slot is handed out again only after
// the stream of its next user waits on the event recorded after its previous
// launch, so a counter is never zeroed or advanced while an earlier launch
// (on any stream) may still read it.  No lock is held across the launch:
// each slot has its own busy flag, taken by compare-and-swap at acquire() and
// dropped at release(), so threads launching on different streams only ever
// contend for one atomic increment (the round-robin cursor).  A thread that
// finds every slot held falls back to the static stride (correct, less
// balanced).
struct QueueRing final : SpareQueue {
    static constexpr uint32_t SLOTS = 256;
    uint32_t *d = nullptr;
    hipEvent_t ev[SLOTS] = {};
    bool recorded[SLOTS] = {};                 // read and written by the slot's holder only
    std::atomic<uint32_t> next{0};
    std::atomic<uint32_t> busy[SLOTS] = {};
    uint32_t *acquire(hipStream_t s, uint32_t *slot) override {
        if (!d) return nullptr;
        for (uint32_t tries = 0; tries < SLOTS; ++tries) {
            const uint32_t i = next.fetch_add(1u, std::memory_order_relaxed) % SLOTS;
            uint32_t free_ = 0u;
            if (!busy[i].compare_exchange_strong(free_, 1u, std::memory_order_acquire)) continue;
            if (recorded[i] && hipStreamWaitEvent(s, ev[i], 0) != hipSuccess) {
                busy[i].store(0u, std::memory_order_release);
                return nullptr;
            }
            *slot = i;
            return d + 16u * i;
        }
        return nullptr;
    }
    void release(hipStream_t s, uint32_t slot) override {
        if (hipEventRecord(ev[slot], s) == hipSuccess) recorded[slot] = true;
        busy[slot].store(0u, std::memory_order_release);
    }
};

struct rt_ctx {
    int device = 0;
    int n_cu = 0;
    // Reclaim stream: a destroyed key set's records are freed here, after
    // the events of their last launches (no host or device-wide sync).
    hipStream_t stream = nullptr;
    uint8_t *d_sbox = nullptr;     // 512 B: S-box || inverse S-box
    // Stream-ordered pool for key records: a per-packet key set per batch
    // (Identity.py:837-846) reuses the memory of the previous one without a
    // hipMalloc/hipFree (both synchronise the device) on the host timeline.
    hipMemPool_t pool = nullptr;
    Stager stagers[N_STAGERS];
    std::atomic<uint32_t> stager_rr{0};
    QueueRing queues;
    // rt_clock_stamps: the launch-clock words the token kernels add to, or null
    std::atomic<unsigned long long *> clk{nullptr};
};

// Takes a free staging lane (or waits for the caller's round-robin one).
struct StageLock {
    Stager *g = nullptr;
    explicit StageLock(rt_ctx *c) {
        const uint32_t start = c->stager_rr.fetch_add(1);
        for (int i = 0; i < N_STAGERS; ++i) {
            Stager &t = c->stagers[(start + i) % N_STAGERS];
            if (t.mu.try_lock()) {
                g = &t;
                return;
            }
        }
        g = &c->stagers[start % N_STAGERS];
        g->mu.lock();
    }
    ~StageLock() { g->mu.unlock(); }
    StageLock(const StageLock &) = delete;
    StageLock &operator=(const StageLock &) = delete;
};

static hipError_t rec_alloc(rt_ctx *c, uint64_t bytes, uint32_t **p, hipStream_t s) {
    *p = nullptr;
    return c->pool ? hipMallocFromPoolAsync((void **)p, bytes, c->pool, s) : hipMallocAsync((void **)p, bytes, s);
}

struct rt_keyset {
    rt_ctx *ctx = nullptr;
    uint32_t key_len = 0, n_keys = 0;
    int nr = 0;
    uint32_t *d_rec = nullptr;
    hipStream_t home = nullptr;    // the stream the records were built on
    hipEvent_t ready = nullptr;    // recorded on `home` after the key setup
    // The last launch on each stream that read the records: destroy orders
    // the free after all of them.
    std::mutex mu;
    std::vector<std::pair<hipStream_t, hipEvent_t>> uses;
};

// Work enqueued on `s` from here on sees the key set's records.
static hipError_t after_setup(const rt_keyset *k, hipStream_t s) {
    return s == k->home ? hipSuccess : hipStreamWaitEvent(s, k->ready, 0);
}
// The launch just enqueued on `s` reads the records.  Entries of other
// streams whose last recorded launch has completed are dropped on the way
// (their event destroyed), so a long-lived key set used from many
// short-lived streams keeps one entry per stream still in flight, and
// rt_keyset_destroy never waits on events of streams that are gone.
static hipError_t note_use(rt_keyset *k, hipStream_t s) {
    std::lock_guard<std::mutex> g(k->mu);
    for (auto &u : k->uses)
        if (u.first == s) return hipEventRecord(u.second, s);
    if (k->uses.size() >= 4) {
        auto done = [](const std::pair<hipStream_t, hipEvent_t> &u) {
            if (hipEventQuery(u.second) != hipSuccess) return false;
            hipEventDestroy(u.second);
            return true;
        };
        k->uses.erase(std::remove_if(k->uses.begin(), k->uses.end(), done), k->uses.end());
    }
    hipEvent_t e = nullptr;
    hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming);
    if (r != hipSuccess) return r;
    k->uses.emplace_back(s, e);
    return hipEventRecord(e, s);
}

static thread_local std::string g_err;

static int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}
static int hip_fail(hipError_t e, const char *what) {
    return fail(RT_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}
#define RT_HIP(call, what)                         \
    do {                                           \
        hipError_t e_ = (call);                    \
        if (e_ != hipSuccess) return hip_fail(e_, what); \
    } while (0)

// S-box from its definition (FIPS-197 §5.1.1): GF(2^8) inverse then affine map.
static void make_sbox(uint8_t s[256], uint8_t inv[256]) {
    uint8_t exp[256], log[256];
    uint8_t x = 1;
    for (int i = 0; i < 255; ++i) {          // generator 3
        exp[i] = x;
        log[x] = (uint8_t)i;
        x = (uint8_t)(x ^ (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1b : 0)));
    }
    for (int v = 0; v < 256; ++v) {
        uint8_t b = v ? exp[(255 - log[v]) % 255] : 0;
        uint8_t r = b;
        for (int i = 0; i < 4; ++i) {
            b = (uint8_t)((b << 1) | (b >> 7));
            r ^= b;
        }
        r ^= 0x63;
        s[v] = r;
        inv[r] = (uint8_t)v;
    }
}

// Device-API streams: the caller's hipStream_t; NULL is HIP's null stream
// (torch's default stream), never the context's private staging stream.
static hipStream_t pick(const rt_ctx *, void *stream) { return (hipStream_t)stream; }

// Device -> host copy on stream s.  A pinned (page-locked, mapped) destination
// is written by GPU stores (launch_store_host: 54 GB/s, and it shares the
// link with a copy-engine H2D at 87 GB/s in total, against 30 GB/s for the
// copy engine's D2H, profiles/r03n_pcie_probe.json); a pageable one goes
// through hipMemcpyAsync.  The store kernel runs on the stream's GPU, so it
// is used only when src is device memory of that GPU (`device`); any other
// source (host memory, another GPU's buffer) takes hipMemcpyAsync, which
// handles every source the copy engine can read.
static bool query(hipPointerAttribute_t *at, const void *p) {
    if (hipPointerGetAttributes(at, p) == hipSuccess) return true;
    (void)hipGetLastError();       // a pageable pointer is an "invalid value" to the query: clear only that
    return false;
}
static hipError_t copy_d2h(void *dst, const void *src, uint64_t bytes, hipStream_t s, int device) {
    if (!bytes) return hipSuccess;
    hipPointerAttribute_t ad, as;
    if (query(&ad, dst) && ad.type == hipMemoryTypeHost && ad.devicePointer && query(&as, src) &&
        as.type == hipMemoryTypeDevice && as.device == device)
        return launch_store_host((uint8_t *)ad.devicePointer, (const uint8_t *)src, bytes, s);
    return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s);
}

static int ensure_work(Stager &g, uint64_t bytes);
static uint8_t *stage(Stager &g, uint64_t bytes);

// One packet per call (Token.encrypt / Token.decrypt): the token kernel reads
// its inputs from the lane's mapped pinned staging buffer and writes its
// outputs there, instead of a copy kernel in, the token kernel, and a store
// kernel out (the runtime's H2D of a small pinned buffer is itself a blit
// kernel, 2.4 us, and the store kernel 3.6 us, each plus its dispatch).  383-B
// packets, one thread: Token.encrypt 57.8 -> 50.1 us, Token.decrypt 45.5 ->
// 38.6 us, 19 100 -> 21 800 calls/s (three runs each,
// profiles/r06_host_direct_ab.txt).  Batches keep the copies (their kernels
// would read every packet across PCIe; not measured).
#ifndef RNSTOK_HOST_DIRECT
#define RNSTOK_HOST_DIRECT 1
#endif

// A key set whose records are allocated and built on stream s.  `build`
// enqueues the kernel(s) that write k->d_rec.
template <class Build>
static rt_keyset *keyset_on(rt_ctx *c, uint32_t key_len, uint32_t n_keys, hipStream_t s, Build build) {
    rt_keyset *k = new rt_keyset();
    k->ctx = c;
    k->key_len = key_len;
    k->n_keys = n_keys;
    k->nr = key_len == 64 ? 14 : 10;
    k->home = s;
    hipError_t e = hipEventCreateWithFlags(&k->ready, hipEventDisableTiming);
    if (e == hipSuccess) e = rec_alloc(c, (uint64_t)n_keys * REC_WORDS * 4, &k->d_rec, s);
    if (e != hipSuccess) {
        fail(RT_E_NOMEM, std::string("key table allocation failed: ") + hipGetErrorString(e));
        if (k->ready) hipEventDestroy(k->ready);
        delete k;
        return nullptr;
    }
    if ((e = build(k)) != hipSuccess || (e = hipEventRecord(k->ready, s)) != hipSuccess) {
        hip_fail(e, "key setup launch");
        hipStreamSynchronize(s);
        hipFreeAsync(k->d_rec, s);
        hipEventDestroy(k->ready);
        delete k;
        return nullptr;
    }
    return k;
}

extern "C" {

int rt_abi_version(void) { return RNSTOK_ABI_VERSION; }
const char *rt_last_error(void) { return g_err.c_str(); }

int rt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

rt_ctx *rt_create(int device) {
    int n = rt_device_count();
    if (device < 0 || device >= n) {
        fail(RT_E_NODEV, "no HIP device " + std::to_string(device) + " (found " + std::to_string(n) + ")");
        return nullptr;
    }
    hipDeviceProp_t prop;
    if (hipSetDevice(device) != hipSuccess || hipGetDeviceProperties(&prop, device) != hipSuccess) {
        fail(RT_E_HIP, "hipGetDeviceProperties failed");
        return nullptr;
    }
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        fail(RT_E_NODEV, std::string("librnstok is built for gfx950, device is ") + prop.gcnArchName);
        return nullptr;
    }
    static std::once_flag once;
    static hipError_t cfg = hipSuccess;
    std::call_once(once, [] { cfg = configure_kernels(); });
    if (cfg != hipSuccess) {
        hip_fail(cfg, "hipFuncSetAttribute(MaxDynamicSharedMemorySize)");
        return nullptr;
    }
    rt_ctx *c = new rt_ctx();
    c->device = device;
    c->n_cu = prop.multiProcessorCount;
    uint8_t tables[512];
    make_sbox(tables, tables + 256);
    bool ok = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess &&
              hipMalloc(&c->d_sbox, 512) == hipSuccess &&
              hipMalloc(&c->queues.d, 64ull * QueueRing::SLOTS) == hipSuccess &&
              hipMemcpy(c->d_sbox, tables, 512, hipMemcpyHostToDevice) == hipSuccess;
    for (uint32_t i = 0; ok && i < QueueRing::SLOTS; ++i)
        ok = hipEventCreateWithFlags(&c->queues.ev[i], hipEventDisableTiming) == hipSuccess;
    for (int i = 0; ok && i < N_STAGERS; ++i)
        ok = hipStreamCreateWithFlags(&c->stagers[i].stream, hipStreamNonBlocking) == hipSuccess;
    if (!ok) {
        fail(RT_E_HIP, "context setup failed");
        rt_destroy(c);
        return nullptr;
    }
    // Key-record pool: keep freed memory for the next key set (no release
    // on synchronisation), reuse across streams through the stream-ordered
    // dependencies.  Without a pool the records come from the device's
    // default one.
    hipMemPoolProps props = {};
    props.allocType = hipMemAllocationTypePinned;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = device;
    if (hipMemPoolCreate(&c->pool, &props) == hipSuccess) {
        uint64_t keep = ~0ull;
        int on = 1;
        hipMemPoolSetAttribute(c->pool, hipMemPoolAttrReleaseThreshold, &keep);
        hipMemPoolSetAttribute(c->pool, hipMemPoolReuseFollowEventDependencies, &on);
        hipMemPoolSetAttribute(c->pool, hipMemPoolReuseAllowOpportunistic, &on);
        hipMemPoolSetAttribute(c->pool, hipMemPoolReuseAllowInternalDependencies, &on);
    } else {
        c->pool = nullptr;
        (void)hipGetLastError();
    }
    return c;
}

void rt_destroy(rt_ctx *c) {
    if (!c) return;
    hipSetDevice(c->device);
    for (auto &g : c->stagers) {
        if (g.stream) hipStreamSynchronize(g.stream);
        hipFree(g.d_work);
        if (g.h_stage) hipHostFree(g.h_stage);
        if (g.stream) hipStreamDestroy(g.stream);
    }
    if (c->stream) hipStreamSynchronize(c->stream);
    hipDeviceSynchronize();            // launches on callers' streams may still use the ring
    hipFree(c->d_sbox);
    hipFree(c->queues.d);
    for (auto &e : c->queues.ev)
        if (e) hipEventDestroy(e);
    if (c->pool) hipMemPoolDestroy(c->pool);
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
}

int rt_num_cus(const rt_ctx *c) { return c ? c->n_cu : 0; }

int rt_plan_uniform(const rt_ctx *c, uint32_t n, uint32_t len, int per_packet_keys, int decrypt) {
    if (!c) return fail(RT_E_INVAL, "rt_plan_uniform: no context");
    return decrypt ? plan_decrypt(n, false, len, per_packet_keys != 0, c->n_cu)
                   : plan_encrypt(n, false, len, per_packet_keys != 0, c->n_cu);
}

uint64_t rt_token_len(uint64_t pt_len) { return 16u + 16u * (pt_len / 16u + 1u) + 32u; }

rt_keyset *rt_keyset_create_device(rt_ctx *c, const uint8_t *d_keys, uint32_t key_len, uint32_t n_keys,
                                   void *stream) {
    if (!c || !d_keys || n_keys == 0) {
        fail(RT_E_INVAL, "rt_keyset_create: null context/keys or zero keys");
        return nullptr;
    }
    if (key_len != 64 && key_len != 32) {   // Token.py:72
        fail(RT_E_INVAL, "Token key must be 128 or 256 bits, not " + std::to_string(key_len * 8));
        return nullptr;
    }
    hipSetDevice(c->device);
    hipStream_t s = pick(c, stream);
    return keyset_on(c, key_len, n_keys, s, [&](rt_keyset *k) {
        return launch_key_setup(d_keys, key_len, n_keys, c->d_sbox, k->d_rec, s);
    });
}

// Host keys: staged through a pinned buffer and a staging lane's workspace;
// the key set is built on that lane's stream and this call does not block
// (later launches on other streams wait on the key set's ready event).
rt_keyset *rt_keyset_create(rt_ctx *c, const uint8_t *keys, uint32_t key_len, uint32_t n_keys) {
    if (!c || !keys || n_keys == 0) {
        fail(RT_E_INVAL, "rt_keyset_create: null context/keys or zero keys");
        return nullptr;
    }
    if (key_len != 64 && key_len != 32) {   // Token.py:72
        fail(RT_E_INVAL, "Token key must be 128 or 256 bits, not " + std::to_string(key_len * 8));
        return nullptr;
    }
    hipSetDevice(c->device);
    const uint64_t bytes = (uint64_t)n_keys * key_len;
    StageLock L(c);
    Stager &g = *L.g;
    if (ensure_work(g, bytes)) return nullptr;
    uint8_t *h = stage(g, bytes);
    hipError_t e;
    if (h) {
        memcpy(h, keys, bytes);
        g.stage_busy = true;
        e = hipMemcpyAsync(g.d_work, h, bytes, hipMemcpyHostToDevice, g.stream);
    } else {
        e = hipMemcpyAsync(g.d_work, keys, bytes, hipMemcpyHostToDevice, g.stream);
    }
    if (e != hipSuccess) {
        hip_fail(e, "key upload failed");
        return nullptr;
    }
    rt_keyset *k = keyset_on(c, key_len, n_keys, g.stream, [&](rt_keyset *ks) {
        return launch_key_setup(g.d_work, key_len, n_keys, c->d_sbox, ks->d_rec, g.stream);
    });
    if (!h) hipStreamSynchronize(g.stream);   // the caller's pageable keys were read in place
    return k;
}

// No synchronisation: the records go back to the pool on the reclaim stream
// once the key setup and the last launch on every stream that used them are
// done.
void rt_keyset_destroy(rt_keyset *k) {
    if (!k) return;
    rt_ctx *c = k->ctx;
    hipSetDevice(c->device);
    hipStreamWaitEvent(c->stream, k->ready, 0);
    {
        std::lock_guard<std::mutex> g(k->mu);
        for (auto &u : k->uses) {
            hipStreamWaitEvent(c->stream, u.second, 0);
            hipEventDestroy(u.second);
        }
        k->uses.clear();
    }
    hipFreeAsync(k->d_rec, c->stream);
    hipEventDestroy(k->ready);
    delete k;
}

uint32_t rt_keyset_size(const rt_keyset *k) { return k ? k->n_keys : 0; }

static int check_keyset(const rt_keyset *k) {
    if (!k || !k->ctx || !k->d_rec) return fail(RT_E_INVAL, "null keyset");
    return RT_OK;
}

static int enc_common(const rt_keyset *k, EncArgs &a, void *stream) {
    int rc = check_keyset(k);
    if (rc) return rc;
    if (a.n == 0) return RT_OK;
    // a uniform batch of empty plaintexts reads no plaintext bytes
    if ((!a.pt && (a.pt_len || a.uni_len)) || !a.iv || !a.tok) return fail(RT_E_INVAL, "rt_encrypt: null buffer");
    a.rec = k->d_rec;
    a.sbox = k->ctx->d_sbox;
    if (unsigned long long *w = k->ctx->clk.load(std::memory_order_acquire)) a.clk = w + 4 * RT_CLOCK_ENCRYPT;
    hipStream_t s = pick(k->ctx, stream);
    RT_HIP(hipSetDevice(k->ctx->device), "hipSetDevice");
    RT_HIP(after_setup(k, s), "wait for key setup");
    RT_HIP(launch_encrypt(a, k->nr, k->ctx->n_cu, &k->ctx->queues, s), "encrypt launch");
    RT_HIP(note_use(const_cast<rt_keyset *>(k), s), "record key set use");
    return RT_OK;
}

static int dec_common(const rt_keyset *k, DecArgs &a, void *stream) {
    int rc = check_keyset(k);
    if (rc) return rc;
    if (a.n == 0) return RT_OK;
    if (!a.tok || !a.pt || !a.out_len || !a.status) return fail(RT_E_INVAL, "rt_decrypt: null buffer");
    a.rec = k->d_rec;
    a.sbox = k->ctx->d_sbox;
    if (unsigned long long *w = k->ctx->clk.load(std::memory_order_acquire)) a.clk = w + 4 * RT_CLOCK_DECRYPT;
    hipStream_t s = pick(k->ctx, stream);
    RT_HIP(hipSetDevice(k->ctx->device), "hipSetDevice");
    RT_HIP(after_setup(k, s), "wait for key setup");
    RT_HIP(launch_decrypt(a, k->nr, k->ctx->n_cu, &k->ctx->queues, s), "decrypt launch");
    RT_HIP(note_use(const_cast<rt_keyset *>(k), s), "record key set use");
    return RT_OK;
}

int rt_encrypt(const rt_keyset *k, const uint8_t *pt, const uint64_t *pt_off, const uint32_t *pt_len,
               const uint32_t *key_idx, const uint8_t *iv, uint8_t *tok, const uint64_t *tok_off, uint32_t n,
               void *stream) {
    if (n && (!pt_off || !pt_len || !tok_off)) return fail(RT_E_INVAL, "rt_encrypt: null offset/length array");
    EncArgs a{};
    a.pt = pt; a.pt_off = pt_off; a.pt_len = pt_len; a.key_idx = key_idx; a.iv = iv;
    a.tok = tok; a.tok_off = tok_off; a.n = n;
    return enc_common(k, a, stream);
}

int rt_encrypt_uniform(const rt_keyset *k, const uint8_t *pt, uint64_t pt_stride, uint32_t pt_len,
                       const uint32_t *key_idx, const uint8_t *iv, uint8_t *tok, uint64_t tok_stride, uint32_t n,
                       void *stream) {
    if (n > 1 && (pt_stride < pt_len || tok_stride < rt_token_len(pt_len)))
        return fail(RT_E_INVAL, "rt_encrypt_uniform: stride smaller than packet/token");
    EncArgs a{};
    a.pt = pt; a.pt_stride = pt_stride; a.uni_len = pt_len; a.key_idx = key_idx; a.iv = iv;
    a.tok = tok; a.tok_stride = tok_stride; a.n = n;
    return enc_common(k, a, stream);
}

int rt_encrypt_interleaved(const rt_keyset *k, const uint8_t *pt, uint32_t pt_len, const uint32_t *key_idx,
                           const uint8_t *iv, uint8_t *tok, uint32_t n, void *stream) {
    EncArgs a{};
    a.pt = pt; a.uni_len = pt_len; a.key_idx = key_idx; a.iv = iv; a.tok = tok; a.n = n; a.ilv = 1;
    return enc_common(k, a, stream);
}

int rt_decrypt_interleaved(const rt_keyset *k, const uint8_t *tok, uint32_t tok_len, const uint32_t *key_idx,
                           uint8_t *pt, uint32_t *pt_len, int32_t *status, uint32_t n, void *stream) {
    if (tok_len < 64u || (tok_len & 15u))
        return fail(RT_E_INVAL, "rt_decrypt_interleaved: token length must be 48 + 16*k, k >= 1");
    DecArgs a{};
    a.tok = tok; a.uni_len = tok_len; a.key_idx = key_idx; a.pt = pt; a.out_len = pt_len; a.status = status; a.n = n;
    a.ilv = 1;
    return dec_common(k, a, stream);
}

int rt_decrypt(const rt_keyset *k, const uint8_t *tok, const uint64_t *tok_off, const uint32_t *tok_len,
               const uint32_t *key_idx, uint8_t *pt, const uint64_t *pt_off, uint32_t *pt_len, int32_t *status,
               uint32_t n, void *stream) {
    if (n && (!tok_off || !tok_len || !pt_off)) return fail(RT_E_INVAL, "rt_decrypt: null offset/length array");
    DecArgs a{};
    a.tok = tok; a.tok_off = tok_off; a.tok_len = tok_len; a.key_idx = key_idx; a.pt = pt; a.pt_off = pt_off;
    a.out_len = pt_len; a.status = status; a.n = n;
    return dec_common(k, a, stream);
}

int rt_decrypt_uniform(const rt_keyset *k, const uint8_t *tok, uint64_t tok_stride, uint32_t tok_len,
                       const uint32_t *key_idx, uint8_t *pt, uint64_t pt_stride, uint32_t *pt_len, int32_t *status,
                       uint32_t n, void *stream) {
    if (n > 1 && (tok_stride < tok_len || (tok_len > 48 && pt_stride < tok_len - 48)))
        return fail(RT_E_INVAL, "rt_decrypt_uniform: stride smaller than token/plaintext");
    DecArgs a{};
    a.tok = tok; a.tok_stride = tok_stride; a.uni_len = tok_len; a.key_idx = key_idx; a.pt = pt;
    a.pt_stride = pt_stride; a.out_len = pt_len; a.status = status; a.n = n;
    return dec_common(k, a, stream);
}

uint64_t rt_workspace_bytes(uint32_t n) { return sort_workspace_bytes(n); }

int rt_encrypt_ex(const rt_keyset *k, const uint8_t *pt, const uint64_t *pt_off, const uint32_t *pt_len,
                  const uint32_t *key_idx, const uint8_t *iv, uint8_t *tok, const uint64_t *tok_off, uint32_t n,
                  uint32_t flags, void *workspace, void *stream) {
    if (n && (!pt_off || !pt_len || !tok_off)) return fail(RT_E_INVAL, "rt_encrypt_ex: null offset/length array");
    if (flags & ~RT_F_SORT_BY_LENGTH) return fail(RT_E_INVAL, "rt_encrypt_ex: unknown flags");
    int rc = check_keyset(k);
    if (rc) return rc;
    EncArgs a{};
    a.pt = pt; a.pt_off = pt_off; a.pt_len = pt_len; a.key_idx = key_idx; a.iv = iv;
    a.tok = tok; a.tok_off = tok_off; a.n = n;
    if ((flags & RT_F_SORT_BY_LENGTH) && n > 1) {
        if (!workspace) return fail(RT_E_INVAL, "rt_encrypt_ex: RT_F_SORT_BY_LENGTH needs a workspace");
        RT_HIP(hipSetDevice(k->ctx->device), "hipSetDevice");
        RT_HIP(launch_length_order(pt_len, n, 0, workspace, &a.order, &a.queue, k->ctx->n_cu, pick(k->ctx, stream)),
               "length order");
    }
    return enc_common(k, a, stream);
}

int rt_decrypt_ex(const rt_keyset *k, const uint8_t *tok, const uint64_t *tok_off, const uint32_t *tok_len,
                  const uint32_t *key_idx, uint8_t *pt, const uint64_t *pt_off, uint32_t *pt_len, int32_t *status,
                  uint32_t n, uint32_t flags, void *workspace, void *stream) {
    if (n && (!tok_off || !tok_len || !pt_off)) return fail(RT_E_INVAL, "rt_decrypt_ex: null offset/length array");
    if (flags & ~RT_F_SORT_BY_LENGTH) return fail(RT_E_INVAL, "rt_decrypt_ex: unknown flags");
    int rc = check_keyset(k);
    if (rc) return rc;
    DecArgs a{};
    a.tok = tok; a.tok_off = tok_off; a.tok_len = tok_len; a.key_idx = key_idx; a.pt = pt; a.pt_off = pt_off;
    a.out_len = pt_len; a.status = status; a.n = n;
    if ((flags & RT_F_SORT_BY_LENGTH) && n > 1) {
        if (!workspace) return fail(RT_E_INVAL, "rt_decrypt_ex: RT_F_SORT_BY_LENGTH needs a workspace");
        RT_HIP(hipSetDevice(k->ctx->device), "hipSetDevice");
        RT_HIP(launch_length_order(tok_len, n, 1, workspace, &a.order, &a.queue, k->ctx->n_cu, pick(k->ctx, stream)),
               "length order");
    }
    return dec_common(k, a, stream);
}

// ---------------------------------------------------------------- host path

static int ensure_work(Stager &g, uint64_t bytes) {
    if (bytes <= g.work_cap) return RT_OK;
    uint64_t cap = std::max<uint64_t>(bytes, g.work_cap * 2);
    cap = (cap + 4095) & ~4095ull;
    if (g.d_work) {
        RT_HIP(hipStreamSynchronize(g.stream), "stream sync");   // queued work may still read the old workspace
        hipFree(g.d_work);
    }
    g.d_work = nullptr;
    g.work_cap = 0;
    if (hipMalloc(&g.d_work, cap) != hipSuccess) return fail(RT_E_NOMEM, "workspace allocation failed");
    g.work_cap = cap;
    return RT_OK;
}

static uint64_t align16(uint64_t x) { return (x + 15) & ~15ull; }

static constexpr uint64_t STAGE_MAX = 8ull << 20;

// The pinned stage for a host call of `bytes`, or null (too large, or the
// pinned allocation failed): the caller then copies from its own pageable
// arrays.  Called with the lane locked.
static uint8_t *stage(Stager &g, uint64_t bytes) {
    if (bytes > STAGE_MAX) return nullptr;
    if (g.stage_busy) {            // a copy from h_stage may still be queued
        if (hipStreamSynchronize(g.stream) != hipSuccess) return nullptr;
        g.stage_busy = false;
    }
    if (bytes > g.stage_cap) {
        const uint64_t cap = std::min<uint64_t>(STAGE_MAX, std::max<uint64_t>({bytes, 2 * g.stage_cap, 64ull << 10}));
        if (g.h_stage) hipHostFree(g.h_stage);
        g.h_stage = nullptr;
        g.stage_cap = 0;
        if (hipHostMalloc(&g.h_stage, cap, hipHostMallocDefault) != hipSuccess) {
            g.h_stage = nullptr;
            return nullptr;
        }
        if (hipHostGetDevicePointer((void **)&g.h_stage_dev, g.h_stage, 0) != hipSuccess) {
            hipHostFree(g.h_stage);
            g.h_stage = g.h_stage_dev = nullptr;
            return nullptr;
        }
        g.stage_cap = cap;
    }
    return g.h_stage;
}

// ----------------------------------------------------------- ratchet trials

int rt_verify_trials(const rt_keyset *k, const uint8_t *tok, const uint64_t *tok_off, const uint32_t *tok_len,
                     const uint32_t *pair_off, const uint32_t *pair_key, uint32_t *first, uint32_t n_tok,
                     uint32_t n_pairs, void *stream) {
    int rc = check_keyset(k);
    if (rc) return rc;
    if (n_tok == 0) return RT_OK;
    if (!tok_off || !tok_len || !pair_off || !first || (n_pairs && (!tok || !pair_key)))
        return fail(RT_E_INVAL, "rt_verify_trials: null argument");
    TrialArgs a{};
    a.rec = k->d_rec; a.tok = tok; a.tok_off = tok_off; a.tok_len = tok_len; a.pair_off = pair_off;
    a.pair_key = pair_key; a.first = first; a.n_tok = n_tok; a.n_pairs = n_pairs;
    hipStream_t s = pick(k->ctx, stream);
    RT_HIP(hipSetDevice(k->ctx->device), "hipSetDevice");
    RT_HIP(after_setup(k, s), "wait for key setup");
    RT_HIP(launch_verify_trials(a, s), "verify trials launch");
    RT_HIP(note_use(const_cast<rt_keyset *>(k), s), "record key set use");
    return RT_OK;
}

int rt_verify_trials_host(const rt_keyset *k, const uint8_t *tok, const uint64_t *tok_off, const uint32_t *tok_len,
                          const uint32_t *pair_off, const uint32_t *pair_key, uint32_t *first, uint32_t n_tok,
                          uint32_t n_pairs) {
    int rc = check_keyset(k);
    if (rc) return rc;
    if (n_tok == 0) return RT_OK;
    if (!tok_off || !tok_len || !pair_off || !first || (n_pairs && !pair_key))
        return fail(RT_E_INVAL, "rt_verify_trials_host: null argument");
    if (pair_off[0] != 0 || pair_off[n_tok] != n_pairs)
        return fail(RT_E_INVAL, "rt_verify_trials_host: pair_off must run from 0 to n_pairs");
    uint64_t tok_ext = 0;
    for (uint32_t t = 0; t < n_tok; ++t) {
        if (pair_off[t + 1] < pair_off[t]) return fail(RT_E_INVAL, "rt_verify_trials_host: pair_off not ascending");
        tok_ext = std::max<uint64_t>(tok_ext, tok_off[t] + tok_len[t]);
    }
    for (uint32_t j = 0; j < n_pairs; ++j)
        if (pair_key[j] >= k->n_keys) return fail(RT_E_INVAL, "pair_key out of range");
    if (tok_ext && !tok) return fail(RT_E_INVAL, "rt_verify_trials_host: null tokens");
    rt_ctx *c = k->ctx;
    StageLock L(c);
    Stager &g = *L.g;
    RT_HIP(hipSetDevice(c->device), "hipSetDevice");
    const uint64_t o_tok = 0, o_to = align16(o_tok + std::max<uint64_t>(tok_ext, 1)), o_tl = align16(o_to + 8ull * n_tok),
                   o_po = align16(o_tl + 4ull * n_tok), o_pk = align16(o_po + 4ull * (n_tok + 1)),
                   o_fi = align16(o_pk + 4ull * std::max<uint32_t>(n_pairs, 1)), total = align16(o_fi + 4ull * n_tok);
    if ((rc = ensure_work(g, total))) return rc;
    uint8_t *w = g.d_work;
    hipStream_t s = g.stream;
    if (tok_ext) RT_HIP(hipMemcpyAsync(w + o_tok, tok, tok_ext, hipMemcpyHostToDevice, s), "H2D tok");
    RT_HIP(hipMemcpyAsync(w + o_to, tok_off, 8ull * n_tok, hipMemcpyHostToDevice, s), "H2D tok_off");
    RT_HIP(hipMemcpyAsync(w + o_tl, tok_len, 4ull * n_tok, hipMemcpyHostToDevice, s), "H2D tok_len");
    RT_HIP(hipMemcpyAsync(w + o_po, pair_off, 4ull * (n_tok + 1), hipMemcpyHostToDevice, s), "H2D pair_off");
    if (n_pairs) RT_HIP(hipMemcpyAsync(w + o_pk, pair_key, 4ull * n_pairs, hipMemcpyHostToDevice, s), "H2D pair_key");
    if ((rc = rt_verify_trials(k, w + o_tok, (const uint64_t *)(w + o_to), (const uint32_t *)(w + o_tl),
                               (const uint32_t *)(w + o_po), (const uint32_t *)(w + o_pk), (uint32_t *)(w + o_fi),
                               n_tok, n_pairs, s)))
        return rc;
    RT_HIP(hipMemcpyAsync(first, w + o_fi, 4ull * n_tok, hipMemcpyDeviceToHost, s), "D2H first");
    RT_HIP(hipStreamSynchronize(s), "stream sync");
    return RT_OK;
}

int rt_encrypt_host(const rt_keyset *k, const uint8_t *pt, const uint64_t *pt_off, const uint32_t *pt_len,
                    const uint32_t *key_idx, const uint8_t *iv, uint8_t *tok, const uint64_t *tok_off, uint32_t n) {
    int rc = check_keyset(k);
    if (rc) return rc;
    if (n == 0) return RT_OK;
    if (!pt_off || !pt_len || !tok_off || !iv || !tok) return fail(RT_E_INVAL, "rt_encrypt_host: null argument");
    uint64_t pt_ext = 0, tok_ext = 0, tok_sum = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (key_idx && key_idx[i] >= k->n_keys) return fail(RT_E_INVAL, "key_idx out of range");
        pt_ext = std::max<uint64_t>(pt_ext, pt_off[i] + pt_len[i]);
        const uint64_t tl = rt_token_len(pt_len[i]);
        tok_ext = std::max<uint64_t>(tok_ext, tok_off[i] + tl);
        tok_sum += tl;
    }
    if (pt_ext && !pt) return fail(RT_E_INVAL, "rt_encrypt_host: null plaintext");
    rt_ctx *c = k->ctx;
    StageLock L(c);
    Stager &g = *L.g;
    RT_HIP(hipSetDevice(c->device), "hipSetDevice");
    // inputs first, the token region last: one copy in, one copy out
    const uint64_t o_pt = 0, o_iv = align16(o_pt + std::max<uint64_t>(pt_ext, 1)), o_po = align16(o_iv + 16ull * n),
                   o_pl = align16(o_po + 8ull * n), o_to = align16(o_pl + 4ull * n), o_ki = align16(o_to + 8ull * n),
                   o_tok = align16(o_ki + (key_idx ? 4ull * n : 0)), total = align16(o_tok + tok_ext);
    if ((rc = ensure_work(g, total))) return rc;
    uint8_t *w = g.d_work;
    hipStream_t s = g.stream;
    const bool gaps = tok_sum != tok_ext;   // gaps between tokens: keep the caller's bytes there
    uint8_t *h = stage(g, total);
    const bool direct = RNSTOK_HOST_DIRECT && h && n == 1;
    if (h) {
        if (pt_ext) memcpy(h + o_pt, pt, pt_ext);
        memcpy(h + o_iv, iv, 16ull * n);
        memcpy(h + o_po, pt_off, 8ull * n);
        memcpy(h + o_pl, pt_len, 4ull * n);
        memcpy(h + o_to, tok_off, 8ull * n);
        if (key_idx) memcpy(h + o_ki, key_idx, 4ull * n);
        if (gaps) memcpy(h + o_tok, tok, tok_ext);
        g.stage_busy = true;
        if (!direct) RT_HIP(hipMemcpyAsync(w, h, gaps ? total : o_tok, hipMemcpyHostToDevice, s), "H2D stage");
    } else {
        if (pt_ext) RT_HIP(hipMemcpyAsync(w + o_pt, pt, pt_ext, hipMemcpyHostToDevice, s), "H2D pt");
        if (gaps) RT_HIP(hipMemcpyAsync(w + o_tok, tok, tok_ext, hipMemcpyHostToDevice, s), "H2D tok");
        RT_HIP(hipMemcpyAsync(w + o_iv, iv, 16ull * n, hipMemcpyHostToDevice, s), "H2D iv");
        RT_HIP(hipMemcpyAsync(w + o_po, pt_off, 8ull * n, hipMemcpyHostToDevice, s), "H2D pt_off");
        RT_HIP(hipMemcpyAsync(w + o_pl, pt_len, 4ull * n, hipMemcpyHostToDevice, s), "H2D pt_len");
        RT_HIP(hipMemcpyAsync(w + o_to, tok_off, 8ull * n, hipMemcpyHostToDevice, s), "H2D tok_off");
        if (key_idx) RT_HIP(hipMemcpyAsync(w + o_ki, key_idx, 4ull * n, hipMemcpyHostToDevice, s), "H2D key_idx");
    }
    if (direct) w = g.h_stage_dev;
    EncArgs a{};
    a.pt = w + o_pt; a.pt_off = (const uint64_t *)(w + o_po); a.pt_len = (const uint32_t *)(w + o_pl);
    a.key_idx = key_idx ? (const uint32_t *)(w + o_ki) : nullptr; a.iv = w + o_iv;
    a.tok = w + o_tok; a.tok_off = (const uint64_t *)(w + o_to); a.n = n;
    if (n == 1) {       // one packet (Token.encrypt): a uniform batch of one, so the latency-shaped kernels apply
        a.pt += pt_off[0]; a.pt_off = nullptr; a.pt_len = nullptr; a.uni_len = pt_len[0];
        a.tok += tok_off[0]; a.tok_off = nullptr;
    }
    if ((rc = enc_common(k, a, s))) return rc;
    if (!direct) RT_HIP(h ? launch_store_host(g.h_stage_dev + o_tok, w + o_tok, tok_ext, s) : copy_d2h(tok, w + o_tok, tok_ext, s, k->ctx->device),
           "D2H tok");
    RT_HIP(hipStreamSynchronize(s), "stream sync");
    g.stage_busy = false;
    if (h) memcpy(tok, h + o_tok, tok_ext);
    return RT_OK;
}

int rt_decrypt_host(const rt_keyset *k, const uint8_t *tok, const uint64_t *tok_off, const uint32_t *tok_len,
                    const uint32_t *key_idx, uint8_t *pt, const uint64_t *pt_off, uint32_t *pt_len, int32_t *status,
                    uint32_t n) {
    int rc = check_keyset(k);
    if (rc) return rc;
    if (n == 0) return RT_OK;
    if (!tok_off || !tok_len || !pt_off || !pt_len || !status) return fail(RT_E_INVAL, "rt_decrypt_host: null argument");
    uint64_t tok_ext = 0, pt_ext = 0, pt_sum = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (key_idx && key_idx[i] >= k->n_keys) return fail(RT_E_INVAL, "key_idx out of range");
        tok_ext = std::max<uint64_t>(tok_ext, tok_off[i] + tok_len[i]);
        const uint64_t pl = tok_len[i] > 48 ? tok_len[i] - 48 : 0;
        pt_ext = std::max<uint64_t>(pt_ext, pt_off[i] + pl);
        pt_sum += pl;
    }
    if ((tok_ext && !tok) || (pt_ext && !pt)) return fail(RT_E_INVAL, "rt_decrypt_host: null buffer");
    rt_ctx *c = k->ctx;
    StageLock L(c);
    Stager &g = *L.g;
    RT_HIP(hipSetDevice(c->device), "hipSetDevice");
    // inputs first, the outputs (plaintexts, lengths, status) last: one copy
    // in, one copy out
    const uint64_t o_tok = 0, o_to = align16(std::max<uint64_t>(tok_ext, 1)), o_tl = align16(o_to + 8ull * n),
                   o_po = align16(o_tl + 4ull * n), o_ki = align16(o_po + 8ull * n),
                   o_pt = align16(o_ki + (key_idx ? 4ull * n : 0)), o_ol = align16(o_pt + std::max<uint64_t>(pt_ext, 1)),
                   o_st = align16(o_ol + 4ull * n), total = align16(o_st + 4ull * n);
    if ((rc = ensure_work(g, total))) return rc;
    uint8_t *w = g.d_work;
    hipStream_t s = g.stream;
    const bool gaps = pt_ext && pt_sum != pt_ext;   // gaps between plaintexts: keep the caller's bytes there
    uint8_t *h = stage(g, total);
    const bool direct = RNSTOK_HOST_DIRECT && h && n == 1;
    if (h) {
        if (tok_ext) memcpy(h + o_tok, tok, tok_ext);
        memcpy(h + o_to, tok_off, 8ull * n);
        memcpy(h + o_tl, tok_len, 4ull * n);
        memcpy(h + o_po, pt_off, 8ull * n);
        if (key_idx) memcpy(h + o_ki, key_idx, 4ull * n);
        if (gaps) memcpy(h + o_pt, pt, pt_ext);
        g.stage_busy = true;
        if (!direct) RT_HIP(hipMemcpyAsync(w, h, gaps ? o_ol : o_pt, hipMemcpyHostToDevice, s), "H2D stage");
    } else {
        if (tok_ext) RT_HIP(hipMemcpyAsync(w + o_tok, tok, tok_ext, hipMemcpyHostToDevice, s), "H2D tok");
        if (gaps) RT_HIP(hipMemcpyAsync(w + o_pt, pt, pt_ext, hipMemcpyHostToDevice, s), "H2D pt");
        RT_HIP(hipMemcpyAsync(w + o_to, tok_off, 8ull * n, hipMemcpyHostToDevice, s), "H2D tok_off");
        RT_HIP(hipMemcpyAsync(w + o_tl, tok_len, 4ull * n, hipMemcpyHostToDevice, s), "H2D tok_len");
        RT_HIP(hipMemcpyAsync(w + o_po, pt_off, 8ull * n, hipMemcpyHostToDevice, s), "H2D pt_off");
        if (key_idx) RT_HIP(hipMemcpyAsync(w + o_ki, key_idx, 4ull * n, hipMemcpyHostToDevice, s), "H2D key_idx");
    }
    if (direct) w = g.h_stage_dev;
    DecArgs a{};
    a.tok = w + o_tok; a.tok_off = (const uint64_t *)(w + o_to); a.tok_len = (const uint32_t *)(w + o_tl);
    a.key_idx = key_idx ? (const uint32_t *)(w + o_ki) : nullptr; a.pt = w + o_pt;
    a.pt_off = (const uint64_t *)(w + o_po); a.out_len = (uint32_t *)(w + o_ol); a.status = (int32_t *)(w + o_st);
    a.n = n;
    if (n == 1) {       // one token (Token.decrypt): a uniform batch of one
        a.tok += tok_off[0]; a.tok_off = nullptr; a.tok_len = nullptr; a.uni_len = tok_len[0];
        a.pt += pt_off[0]; a.pt_off = nullptr;
    }
    if ((rc = dec_common(k, a, s))) return rc;
    if (h) {
        if (!direct) RT_HIP(launch_store_host(g.h_stage_dev + o_pt, w + o_pt, total - o_pt, s), "D2H stage");
        RT_HIP(hipStreamSynchronize(s), "stream sync");
        g.stage_busy = false;
        if (pt_ext) memcpy(pt, h + o_pt, pt_ext);
        memcpy(pt_len, h + o_ol, 4ull * n);
        memcpy(status, h + o_st, 4ull * n);
        return RT_OK;
    }
    if (pt_ext) RT_HIP(copy_d2h(pt, w + o_pt, pt_ext, s, k->ctx->device), "D2H pt");
    RT_HIP(copy_d2h(pt_len, w + o_ol, 4ull * n, s, k->ctx->device), "D2H pt_len");
    RT_HIP(copy_d2h(status, w + o_st, 4ull * n, s, k->ctx->device), "D2H status");
    RT_HIP(hipStreamSynchronize(s), "stream sync");
    return RT_OK;
}


// ------------------------------------------------------------------ wire --

static_assert(sizeof(rt_packet_fields) == 96, "rt_packet_fields layout");

uint64_t rt_hdlc_frame_workspace_bytes(uint32_t n) { return hdlc_frame_workspace_bytes(n); }
uint64_t rt_hdlc_deframe_workspace_bytes(uint64_t len) { return hdlc_deframe_workspace_bytes(len); }

int rt_hdlc_frame(rt_ctx *c, const uint8_t *pkt, const uint64_t *pkt_off, const uint32_t *pkt_len, uint32_t n,
                  uint8_t *out, uint64_t *frame_off, void *workspace, void *stream) {
    if (!c) return fail(RT_E_INVAL, "null context");
    if (!frame_off) return fail(RT_E_INVAL, "rt_hdlc_frame: null frame_off");
    if (n == 0) return RT_OK;
    if (!pkt || !pkt_off || !pkt_len || !out || !workspace) return fail(RT_E_INVAL, "rt_hdlc_frame: null buffer");
    RT_HIP(hipSetDevice(c->device), "hipSetDevice");
    RT_HIP(launch_hdlc_frame(pkt, pkt_off, pkt_len, n, out, frame_off, workspace, pick(c, stream)), "hdlc frame");
    return RT_OK;
}

static int deframe_common(rt_ctx *c, const uint8_t *buf, uint64_t len, uint32_t hw_mtu, uint32_t ifac_size,
                          uint8_t *out, uint64_t *frame_off, uint32_t *frame_len, int32_t *status, uint64_t *counts,
                          uint64_t max_pairs, void *workspace, void *stream, uint32_t line_phase) {
    if (!c) return fail(RT_E_INVAL, "null context");
    if (!counts || !workspace) return fail(RT_E_INVAL, "rt_hdlc_deframe: null counts/workspace");
    if (len && (!buf || !out)) return fail(RT_E_INVAL, "rt_hdlc_deframe: null buffer");
    if (max_pairs && (!frame_off || !frame_len || !status)) return fail(RT_E_INVAL, "rt_hdlc_deframe: null frame arrays");
    RT_HIP(hipSetDevice(c->device), "hipSetDevice");
    RT_HIP(launch_hdlc_deframe(buf, len, hw_mtu, ifac_size, out, frame_off, frame_len, status, counts, max_pairs,
                               workspace, pick(c, stream), line_phase),
           "hdlc deframe");
    return RT_OK;
}

int rt_hdlc_deframe(rt_ctx *c, const uint8_t *buf, uint64_t len, uint32_t hw_mtu, uint32_t ifac_size, uint8_t *out,
                    uint64_t *frame_off, uint32_t *frame_len, int32_t *status, uint64_t *counts, uint64_t max_pairs,
                    void *workspace, void *stream) {
    return deframe_common(c, buf, len, hw_mtu, ifac_size, out, frame_off, frame_len, status, counts, max_pairs,
                          workspace, stream, 0xFFFFFFFFu);
}

int rt_hdlc_deframe_slots(rt_ctx *c, const uint8_t *buf, uint64_t len, uint32_t hw_mtu, uint32_t ifac_size,
                          uint32_t line_phase, uint8_t *out, uint64_t *frame_off, uint32_t *frame_len, int32_t *status,
                          uint64_t *counts, uint64_t max_pairs, void *workspace, void *stream) {
    if (line_phase >= 128u) return fail(RT_E_INVAL, "rt_hdlc_deframe_slots: line_phase must be < 128");
    return deframe_common(c, buf, len, hw_mtu, ifac_size, out, frame_off, frame_len, status, counts, max_pairs,
                          workspace, stream, line_phase);
}

static bool overlaps(const void *a, const void *b, uint64_t a_bytes, uint64_t b_bytes = 0) {
    const uintptr_t x = (uintptr_t)a, y = (uintptr_t)b;
    return x < y + (b_bytes ? b_bytes : a_bytes) && y < x + a_bytes;
}

uint64_t rt_frames_compact_workspace_bytes(uint64_t max_pairs) { return frames_compact_workspace_bytes(max_pairs); }

int rt_frames_compact(rt_ctx *c, const uint64_t *frame_off, const uint32_t *frame_len, const int32_t *status,
                      const uint64_t *counts, uint64_t max_pairs, uint64_t *f_off, uint32_t *f_len,
                      int64_t *frame_pair, int64_t *n_frames, void *workspace, void *stream) {
    if (!c) return fail(RT_E_INVAL, "null context");
    if (!counts || !n_frames) return fail(RT_E_INVAL, "rt_frames_compact: null counts/n_frames");
    if (max_pairs && (!frame_off || !frame_len || !status || !f_off || !f_len || !frame_pair || !workspace))
        return fail(RT_E_INVAL, "rt_frames_compact: null buffer");
    // k_compact_write reads frame_off[k] / frame_len[k] while other threads
    // write f_off[r] / f_len[r] for r <= k: in-place compaction would race
    if (max_pairs && (overlaps(f_off, frame_off, 8 * max_pairs) || overlaps(f_len, frame_len, 4 * max_pairs) ||
                      overlaps(f_off, frame_len, 8 * max_pairs, 4 * max_pairs) ||
                      overlaps(f_len, frame_off, 4 * max_pairs, 8 * max_pairs)))
        return fail(RT_E_INVAL, "rt_frames_compact: outputs must not overlap the frame arrays");
    RT_HIP(hipSetDevice(c->device), "hipSetDevice");
    RT_HIP(launch_frames_compact(frame_off, frame_len, status, counts, max_pairs, f_off, f_len, frame_pair, n_frames,
                                 workspace, pick(c, stream)),
           "frames compact");
    return RT_OK;
}

int rt_ifac_mask(rt_ctx *c, const uint8_t *pkt, const uint64_t *pkt_off, const uint32_t *pkt_len, const uint8_t *ifac,
                 uint32_t ifac_size, const uint8_t *ifac_key, uint32_t key_len, uint8_t *out, const uint64_t *out_off,
                 uint32_t n, void *stream) {
    if (!c) return fail(RT_E_INVAL, "null context");
    if (key_len > 64) return fail(RT_E_INVAL, "rt_ifac_mask: ifac_key longer than 64 bytes");
    if (ifac_size == 0 || ifac_size > 64) return fail(RT_E_INVAL, "rt_ifac_mask: ifac_size must be 1..64");
    if (n == 0) return RT_OK;
    if (!pkt || !pkt_off || !pkt_len || !ifac || !out || !out_off || (key_len && !ifac_key))
        return fail(RT_E_INVAL, "rt_ifac_mask: null buffer");
    IfacArgs a{pkt, pkt_off, pkt_len, const_cast<uint8_t *>(ifac), ifac_size, ifac_key, key_len, out, out_off,
               nullptr, nullptr, n};
    RT_HIP(hipSetDevice(c->device), "hipSetDevice");
    RT_HIP(launch_ifac(a, true, pick(c, stream)), "ifac mask");
    return RT_OK;
}

int rt_ifac_unmask(rt_ctx *c, const uint8_t *pkt, const uint64_t *pkt_off, const uint32_t *pkt_len, uint32_t ifac_size,
                   const uint8_t *ifac_key, uint32_t key_len, uint8_t *ifac_out, uint8_t *out, const uint64_t *out_off,
                   int32_t *status, uint32_t *out_len, uint32_t n, void *stream) {
    if (!c) return fail(RT_E_INVAL, "null context");
    if (key_len > 64) return fail(RT_E_INVAL, "rt_ifac_unmask: ifac_key longer than 64 bytes");
    if (ifac_size == 0 || ifac_size > 64) return fail(RT_E_INVAL, "rt_ifac_unmask: ifac_size must be 1..64");
    if (n == 0) return RT_OK;
    if (!pkt || !pkt_off || !pkt_len || !ifac_out || !out || !out_off || !status || (key_len && !ifac_key))
        return fail(RT_E_INVAL, "rt_ifac_unmask: null buffer");
    IfacArgs a{pkt, pkt_off, pkt_len, ifac_out, ifac_size, ifac_key, key_len, out, out_off, status, out_len, n};
    RT_HIP(hipSetDevice(c->device), "hipSetDevice");
    RT_HIP(launch_ifac(a, false, pick(c, stream)), "ifac unmask");
    return RT_OK;
}

int rt_packet_unpack(rt_ctx *c, const uint8_t *pkt, const uint64_t *pkt_off, const uint32_t *pkt_len,
                     rt_packet_fields *fields, uint32_t n, void *stream) {
    if (!c) return fail(RT_E_INVAL, "null context");
    if (n == 0) return RT_OK;
    if (!pkt || !pkt_off || !pkt_len || !fields) return fail(RT_E_INVAL, "rt_packet_unpack: null buffer");
    RT_HIP(hipSetDevice(c->device), "hipSetDevice");
    RT_HIP(launch_unpack(pkt, pkt_off, pkt_len, fields, n, pick(c, stream)), "packet unpack");
    return RT_OK;
}

int rt_token_spans(rt_ctx *c, const rt_packet_fields *fields, const uint64_t *pkt_off, uint32_t n, uint64_t *tok_off,
                   uint32_t *tok_len, void *stream) {
    if (!c) return fail(RT_E_INVAL, "null context");
    if (n == 0) return RT_OK;
    if (!fields || !pkt_off || !tok_off || !tok_len) return fail(RT_E_INVAL, "rt_token_spans: null buffer");
    RT_HIP(hipSetDevice(c->device), "hipSetDevice");
    RT_HIP(launch_token_spans(fields, pkt_off, n, tok_off, tok_len, pick(c, stream)), "token spans");
    return RT_OK;
}

int rt_packet_pack_headers(rt_ctx *c, const uint8_t *flags, const uint8_t *hops, const uint8_t *transport_id,
                           const uint8_t *destination_hash, const uint8_t *context, uint8_t *out,
                           const uint64_t *out_off, uint32_t n, void *stream) {
    if (!c) return fail(RT_E_INVAL, "null context");
    if (n == 0) return RT_OK;
    if (!flags || !destination_hash || !context || !out || !out_off)
        return fail(RT_E_INVAL, "rt_packet_pack_headers: null buffer");
    PackArgs a{flags, hops, context, destination_hash, transport_id, out, out_off, n};
    RT_HIP(hipSetDevice(c->device), "hipSetDevice");
    RT_HIP(launch_pack_headers(a, pick(c, stream)), "pack headers");
    return RT_OK;
}

// --------------------------------------------------------- Resource hashmap --

int rt_map_hashes(rt_ctx *c, const uint8_t *data, const uint64_t *part_off, const uint32_t *part_len, uint64_t size,
                  uint32_t sdu, const uint8_t *salts, uint32_t salt_len, const uint32_t *part_res, uint32_t n_res,
                  uint32_t guard, uint8_t *map_hashes, uint32_t *first_collision, uint32_t n_parts, void *stream) {
    if (!c) return fail(RT_E_INVAL, "null context");
    if (n_parts == 0) return RT_OK;
    if (!data || !map_hashes) return fail(RT_E_INVAL, "rt_map_hashes: null data or output");
    if ((part_off == nullptr) != (part_len == nullptr))
        return fail(RT_E_INVAL, "rt_map_hashes: part_off and part_len go together");
    if (!part_off) {
        if (sdu == 0 || (size + sdu - 1) / sdu != n_parts)
            return fail(RT_E_INVAL, "rt_map_hashes: n_parts must be ceil(size / sdu)");
        if (part_res) return fail(RT_E_INVAL, "rt_map_hashes: uniform segmentation is one resource");
    }
    if (salt_len && !salts) return fail(RT_E_INVAL, "rt_map_hashes: null salts");
    if (n_res == 0) n_res = 1;
    MapArgs m{};
    m.data = data; m.part_off = part_off; m.part_len = part_len; m.size = size; m.sdu = sdu;
    m.salts = salts; m.salt_len = salts ? salt_len : 0; m.part_res = part_res; m.n_res = n_res; m.guard = guard;
    m.out = map_hashes; m.first_collision = first_collision; m.n_parts = n_parts;
    RT_HIP(hipSetDevice(c->device), "hipSetDevice");
    RT_HIP(launch_map_hashes(m, pick(c, stream)), "map hash launch");
    return RT_OK;
}

int rt_resource_hashmap_host(rt_ctx *c, const uint8_t *data, uint64_t size, uint32_t sdu, const uint8_t *random_hash,
                             uint32_t rh_len, uint32_t guard, uint8_t *hashmap, uint32_t *first_collision) {
    if (!c) return fail(RT_E_INVAL, "null context");
    if (sdu == 0) return fail(RT_E_INVAL, "rt_resource_hashmap_host: sdu must be > 0");
    const uint64_t parts = (size + sdu - 1) / sdu;
    if (parts > 0xffffffffull) return fail(RT_E_INVAL, "rt_resource_hashmap_host: too many parts");
    if (first_collision) *first_collision = 0xffffffffu;
    if (parts == 0) return RT_OK;
    if (!data || !hashmap || (rh_len && !random_hash)) return fail(RT_E_INVAL, "rt_resource_hashmap_host: null buffer");
    const uint64_t o_data = 0, o_salt = align16(size), o_out = align16(o_salt + rh_len),
                   o_col = align16(o_out + 4 * parts), total = align16(o_col + 4);
    StageLock L(c);
    Stager &g = *L.g;
    RT_HIP(hipSetDevice(c->device), "hipSetDevice");
    int rc = ensure_work(g, total);
    if (rc) return rc;
    uint8_t *w = g.d_work;
    hipStream_t s = g.stream;
    RT_HIP(hipMemcpyAsync(w + o_data, data, size, hipMemcpyHostToDevice, s), "H2D data");
    if (rh_len) RT_HIP(hipMemcpyAsync(w + o_salt, random_hash, rh_len, hipMemcpyHostToDevice, s), "H2D salt");
    MapArgs m{};
    m.data = w + o_data; m.size = size; m.sdu = sdu; m.salts = w + o_salt; m.salt_len = rh_len; m.n_res = 1;
    m.guard = guard; m.out = w + o_out; m.first_collision = (uint32_t *)(w + o_col); m.n_parts = (uint32_t)parts;
    RT_HIP(launch_map_hashes(m, s), "map hash launch");
    RT_HIP(hipMemcpyAsync(hashmap, w + o_out, 4 * parts, hipMemcpyDeviceToHost, s), "D2H hashmap");
    uint32_t col = 0xffffffffu;
    RT_HIP(hipMemcpyAsync(&col, w + o_col, 4, hipMemcpyDeviceToHost, s), "D2H collision");
    RT_HIP(hipStreamSynchronize(s), "stream sync");
    if (first_collision) *first_collision = col;
    return RT_OK;
}

// ------------------------------------------------------------------ HKDF --

static int hkdf_check(rt_ctx *c, const uint8_t *ikm, uint32_t ikm_len, const uint8_t *context, uint32_t context_len,
                      uint32_t length) {
    if (!c) return fail(RT_E_INVAL, "null context");
    if (length < 1) return fail(RT_E_INVAL, "Invalid output key length");          // HKDF.py:40-41
    if (ikm_len && !ikm) return fail(RT_E_INVAL, "Cannot derive key from empty input material");   // HKDF.py:43-44
    if (context_len && !context) return fail(RT_E_INVAL, "rt_hkdf: null context bytes");
    return RT_OK;
}

static HkdfArgs hkdf_args(const uint8_t *ikm, uint64_t ikm_stride, uint32_t ikm_len, const uint8_t *salt,
                          uint64_t salt_stride, uint32_t salt_len, const uint8_t *context, uint32_t context_len,
                          uint8_t *out, uint64_t out_stride, uint32_t length, uint32_t n) {
    HkdfArgs a{};
    a.ikm = ikm; a.ikm_stride = ikm_stride; a.ikm_len = ikm_len;
    a.salt = salt_len ? salt : nullptr; a.salt_stride = salt_stride; a.salt_len = salt ? salt_len : 0;
    a.context = context_len ? context : nullptr; a.context_len = context ? context_len : 0;
    a.out = out; a.out_stride = out_stride; a.length = length; a.n = n;
    return a;
}

int rt_hkdf(rt_ctx *c, const uint8_t *ikm, uint64_t ikm_stride, uint32_t ikm_len, const uint8_t *salt,
            uint64_t salt_stride, uint32_t salt_len, const uint8_t *context, uint32_t context_len, uint8_t *out,
            uint64_t out_stride, uint32_t length, uint32_t n, void *stream) {
    int rc = hkdf_check(c, ikm, ikm_len, context, context_len, length);
    if (rc || n == 0) return rc;
    if (!out) return fail(RT_E_INVAL, "rt_hkdf: null output");
    RT_HIP(hipSetDevice(c->device), "hipSetDevice");
    const HkdfArgs a = hkdf_args(ikm, ikm_stride, ikm_len, salt, salt_stride, salt_len, context, context_len, out,
                                 out_stride, length, n);
    RT_HIP(launch_hkdf(a, pick(c, stream)), "hkdf launch");
    return RT_OK;
}

int rt_hkdf_host(rt_ctx *c, const uint8_t *ikm, uint64_t ikm_stride, uint32_t ikm_len, const uint8_t *salt,
                 uint64_t salt_stride, uint32_t salt_len, const uint8_t *context, uint32_t context_len, uint8_t *out,
                 uint64_t out_stride, uint32_t length, uint32_t n) {
    int rc = hkdf_check(c, ikm, ikm_len, context, context_len, length);
    if (rc || n == 0) return rc;
    if (!out) return fail(RT_E_INVAL, "rt_hkdf: null output");
    if (!salt) salt_len = 0;
    if (!context) context_len = 0;
    // packed copies on the device: ikm n x ikm_len, salt n x salt_len, context, out n x length
    const uint64_t b_ikm = (uint64_t)n * ikm_len, b_salt = (salt_stride ? (uint64_t)n : 1ull) * salt_len,
                   b_out = (uint64_t)n * length;   // salt_stride 0: one shared salt row
    const uint64_t o_ikm = 0, o_salt = align16(o_ikm + b_ikm), o_ctx = align16(o_salt + b_salt),
                   o_out = align16(o_ctx + context_len), total = align16(o_out + b_out);
    StageLock L(c);
    Stager &g = *L.g;
    RT_HIP(hipSetDevice(c->device), "hipSetDevice");
    if ((rc = ensure_work(g, total))) return rc;
    uint8_t *w = g.d_work;
    hipStream_t s = g.stream;
    if (b_ikm)
        RT_HIP(hipMemcpy2DAsync(w + o_ikm, ikm_len, ikm, ikm_stride, ikm_len, n, hipMemcpyHostToDevice, s), "H2D ikm");
    if (b_salt)
        RT_HIP(hipMemcpy2DAsync(w + o_salt, salt_len, salt, salt_stride ? salt_stride : salt_len, salt_len,
                                salt_stride ? n : 1u, hipMemcpyHostToDevice, s),
               "H2D salt");
    if (context_len) RT_HIP(hipMemcpyAsync(w + o_ctx, context, context_len, hipMemcpyHostToDevice, s), "H2D context");
    const HkdfArgs a = hkdf_args(w + o_ikm, ikm_len, ikm_len, b_salt ? w + o_salt : nullptr, salt_stride ? salt_len : 0, salt_len,
                                 context_len ? w + o_ctx : nullptr, context_len, w + o_out, length, length, n);
    RT_HIP(launch_hkdf(a, s), "hkdf launch");
    RT_HIP(hipMemcpy2DAsync(out, out_stride, w + o_out, length, length, n, hipMemcpyDeviceToHost, s), "D2H out");
    RT_HIP(hipStreamSynchronize(s), "stream sync");
    return RT_OK;
}

rt_keyset *rt_keyset_create_hkdf(rt_ctx *c, const uint8_t *ikm, uint64_t ikm_stride, uint32_t ikm_len,
                                 const uint8_t *salt, uint64_t salt_stride, uint32_t salt_len,
                                 const uint8_t *context, uint32_t context_len, uint32_t key_len, uint32_t n,
                                 void *stream) {
    if (hkdf_check(c, ikm, ikm_len, context, context_len, key_len)) return nullptr;
    if (n == 0) {
        fail(RT_E_INVAL, "rt_keyset_create_hkdf: zero keys");
        return nullptr;
    }
    if (key_len != 64 && key_len != 32) {   // Token.py:72
        fail(RT_E_INVAL, "Token key must be 128 or 256 bits, not " + std::to_string(key_len * 8));
        return nullptr;
    }
    hipSetDevice(c->device);
    hipStream_t s = pick(c, stream);
    const HkdfArgs a = hkdf_args(ikm, ikm_stride, ikm_len, salt, salt_stride, salt_len, context, context_len, nullptr,
                                 key_len, key_len, n);
    return keyset_on(c, key_len, n, s, [&](rt_keyset *k) {
        // one launch: derive each key in registers and build its record
        hipError_t e = launch_hkdf_key_setup(a, c->d_sbox, k->d_rec, c->n_cu, s);
        if (e != hipErrorNotSupported) return e;
        // other shapes (context, long or unaligned ikm/salt): HKDF into a
        // stream-ordered temporary, then the key setup
        uint8_t *d_keys = nullptr;
        if ((e = hipMallocAsync((void **)&d_keys, (uint64_t)n * key_len, s)) != hipSuccess) return e;
        HkdfArgs t = a;
        t.out = d_keys;
        e = launch_hkdf(t, s);
        if (e == hipSuccess) e = launch_key_setup(d_keys, key_len, n, c->d_sbox, k->d_rec, s);
        hipFreeAsync(d_keys, s);     // freed after the key setup has consumed it
        return e;
    });
}

// ------------------------------------------------------------- verify_hmac

static int verify_common(const rt_keyset *k, VerifyArgs &a, void *stream) {
    int rc = check_keyset(k);
    if (rc) return rc;
    if (a.n == 0) return RT_OK;
    if (!a.status) return fail(RT_E_INVAL, "rt_verify: null status");
    a.rec = k->d_rec;
    hipStream_t s = pick(k->ctx, stream);
    RT_HIP(hipSetDevice(k->ctx->device), "hipSetDevice");
    RT_HIP(after_setup(k, s), "wait for key setup");
    RT_HIP(launch_verify(a, s), "verify launch");
    RT_HIP(note_use(const_cast<rt_keyset *>(k), s), "record key set use");
    return RT_OK;
}

int rt_verify(const rt_keyset *k, const uint8_t *tok, const uint64_t *tok_off, const uint32_t *tok_len,
              const uint32_t *key_idx, int32_t *status, uint32_t n, void *stream) {
    if (n && (!tok_off || !tok_len)) return fail(RT_E_INVAL, "rt_verify: null offset/length array");
    VerifyArgs a{};
    a.tok = tok; a.tok_off = tok_off; a.tok_len = tok_len; a.key_idx = key_idx; a.status = status; a.n = n;
    return verify_common(k, a, stream);
}

int rt_verify_host(const rt_keyset *k, const uint8_t *tok, const uint64_t *tok_off, const uint32_t *tok_len,
                   const uint32_t *key_idx, int32_t *status, uint32_t n) {
    int rc = check_keyset(k);
    if (rc) return rc;
    if (n == 0) return RT_OK;
    if (!tok_off || !tok_len || !status) return fail(RT_E_INVAL, "rt_verify_host: null argument");
    uint64_t tok_ext = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (key_idx && key_idx[i] >= k->n_keys) return fail(RT_E_INVAL, "key_idx out of range");
        tok_ext = std::max<uint64_t>(tok_ext, tok_off[i] + tok_len[i]);
    }
    if (tok_ext && !tok) return fail(RT_E_INVAL, "rt_verify_host: null tokens");
    rt_ctx *c = k->ctx;
    StageLock L(c);
    Stager &g = *L.g;
    RT_HIP(hipSetDevice(c->device), "hipSetDevice");
    const uint64_t o_tok = 0, o_to = align16(std::max<uint64_t>(tok_ext, 1)), o_tl = align16(o_to + 8ull * n),
                   o_ki = align16(o_tl + 4ull * n), o_st = align16(o_ki + (key_idx ? 4ull * n : 0)),
                   total = align16(o_st + 4ull * n);
    if ((rc = ensure_work(g, total))) return rc;
    uint8_t *w = g.d_work;
    hipStream_t s = g.stream;
    uint8_t *h = stage(g, total);
    if (h) {
        if (tok_ext) memcpy(h + o_tok, tok, tok_ext);
        memcpy(h + o_to, tok_off, 8ull * n);
        memcpy(h + o_tl, tok_len, 4ull * n);
        if (key_idx) memcpy(h + o_ki, key_idx, 4ull * n);
        g.stage_busy = true;
        RT_HIP(hipMemcpyAsync(w, h, o_st, hipMemcpyHostToDevice, s), "H2D stage");
    } else {
        if (tok_ext) RT_HIP(hipMemcpyAsync(w + o_tok, tok, tok_ext, hipMemcpyHostToDevice, s), "H2D tok");
        RT_HIP(hipMemcpyAsync(w + o_to, tok_off, 8ull * n, hipMemcpyHostToDevice, s), "H2D tok_off");
        RT_HIP(hipMemcpyAsync(w + o_tl, tok_len, 4ull * n, hipMemcpyHostToDevice, s), "H2D tok_len");
        if (key_idx) RT_HIP(hipMemcpyAsync(w + o_ki, key_idx, 4ull * n, hipMemcpyHostToDevice, s), "H2D key_idx");
    }
    VerifyArgs a{};
    a.tok = w + o_tok; a.tok_off = (const uint64_t *)(w + o_to); a.tok_len = (const uint32_t *)(w + o_tl);
    a.key_idx = key_idx ? (const uint32_t *)(w + o_ki) : nullptr; a.status = (int32_t *)(w + o_st); a.n = n;
    if ((rc = verify_common(k, a, s))) return rc;
    RT_HIP(h ? launch_store_host(g.h_stage_dev + o_st, w + o_st, 4ull * n, s) : copy_d2h(status, w + o_st, 4ull * n, s, k->ctx->device),
           "D2H status");
    RT_HIP(hipStreamSynchronize(s), "stream sync");
    g.stage_busy = false;
    if (h) memcpy(status, h + o_st, 4ull * n);
    return RT_OK;
}

// ------------------------------------------------------------------ memory

void *rt_device_alloc(rt_ctx *c, uint64_t bytes) {
    if (!c) return nullptr;
    void *p = nullptr;
    hipSetDevice(c->device);
    if (hipMalloc(&p, bytes ? bytes : 1) != hipSuccess) {
        fail(RT_E_NOMEM, "hipMalloc failed");
        return nullptr;
    }
    return p;
}
void rt_device_free(rt_ctx *c, void *p) {
    if (c) hipSetDevice(c->device);
    hipFree(p);
}
void *rt_host_alloc(uint64_t bytes) {
    void *p = nullptr;
    if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) {
        fail(RT_E_NOMEM, "hipHostMalloc failed");
        return nullptr;
    }
    return p;
}
void rt_host_free(void *p) { hipHostFree(p); }
int rt_memcpy_h2d(rt_ctx *c, void *dst, const void *src, uint64_t bytes, void *stream) {
    if (!c) return fail(RT_E_INVAL, "null context");
    RT_HIP(hipSetDevice(c->device), "hipSetDevice");
    RT_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, pick(c, stream)), "H2D");
    return RT_OK;
}
int rt_memcpy_d2h(rt_ctx *c, void *dst, const void *src, uint64_t bytes, void *stream) {
    if (!c) return fail(RT_E_INVAL, "null context");
    RT_HIP(hipSetDevice(c->device), "hipSetDevice");
    RT_HIP(copy_d2h(dst, src, bytes, pick(c, stream), c->device), "D2H");
    return RT_OK;
}
int rt_memcpy_d2h_upto(rt_ctx *c, void *dst, const void *src, uint64_t max_bytes, const uint64_t *d_bytes,
                       void *stream) {
    if (!c || !dst || !src || !d_bytes) return fail(RT_E_INVAL, "rt_memcpy_d2h_upto: null argument");
    RT_HIP(hipSetDevice(c->device), "hipSetDevice");
    hipPointerAttribute_t ad, as, an;
    if (!(query(&ad, dst) && ad.type == hipMemoryTypeHost && ad.devicePointer && query(&as, src) &&
          as.type == hipMemoryTypeDevice && as.device == c->device))
        return fail(RT_E_INVAL, "rt_memcpy_d2h_upto: dst must be pinned host memory and src device memory of the "
                                "context's GPU");
    if (!(query(&an, d_bytes) && an.type == hipMemoryTypeDevice && an.device == c->device))
        return fail(RT_E_INVAL, "rt_memcpy_d2h_upto: d_bytes must be device memory of the context's GPU");
    RT_HIP(launch_store_host((uint8_t *)ad.devicePointer, (const uint8_t *)src, max_bytes, pick(c, stream), d_bytes),
           "D2H");
    return RT_OK;
}
int rt_clock_stamps(rt_ctx *c, uint64_t *acc) {
    if (!c) return fail(RT_E_INVAL, "null context");
    if (acc) {
        RT_HIP(hipSetDevice(c->device), "hipSetDevice");
        hipPointerAttribute_t at;
        if (((uintptr_t)acc & 7u) || !(query(&at, acc) && at.type == hipMemoryTypeDevice && at.device == c->device))
            return fail(RT_E_INVAL, "rt_clock_stamps: acc must be 8-byte aligned device memory of the context's GPU");
    }
    c->clk.store((unsigned long long *)acc, std::memory_order_release);
    return RT_OK;
}
int rt_stream_sync(rt_ctx *c, void *stream) {
    if (!c) return fail(RT_E_INVAL, "null context");
    RT_HIP(hipSetDevice(c->device), "hipSetDevice");
    RT_HIP(hipStreamSynchronize(pick(c, stream)), "stream sync");
    return RT_OK;
}

}  // extern "C"
