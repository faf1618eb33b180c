// token_launch.h — internal interface between the C-ABI layer and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rnstok {

struct EncArgs {
    const uint32_t *rec;        // key records (REC_WORDS each)
    const uint8_t *sbox;        // 256 B S-box || 256 B inverse S-box (device)
    const uint8_t *pt;
    const uint64_t *pt_off;     // null -> i * pt_stride
    uint64_t pt_stride;
    const uint32_t *pt_len;     // null -> uni_len
    uint32_t uni_len;
    const uint32_t *key_idx;    // null -> key 0
    const uint8_t *iv;
    uint8_t *tok;
    const uint64_t *tok_off;    // null -> i * tok_stride
    uint64_t tok_stride;
    const uint32_t *order;      // null -> lane i handles packet i; else packet order[i]
    uint32_t *queue;            // null -> static grid stride; else a zeroed chunk counter (sorted batches)
    uint32_t n;
    uint32_t ilv;               // 1: unit-interleaved layout (16-B unit u of packet p at 16*(u*n + p)), uniform
    unsigned long long *clk;    // null, or this kernel class's 4 launch-clock words (rt_clock_stamps)
};

struct DecArgs {
    const uint32_t *rec;
    const uint8_t *sbox;
    const uint8_t *tok;
    const uint64_t *tok_off;
    uint64_t tok_stride;
    const uint32_t *tok_len;
    uint32_t uni_len;
    const uint32_t *key_idx;
    uint8_t *pt;
    const uint64_t *pt_off;
    uint64_t pt_stride;
    uint32_t *out_len;
    int32_t *status;
    const uint32_t *order;      // null -> lane i handles token i; else token order[i]
    uint32_t *queue;            // as EncArgs::queue
    uint32_t n;
    uint32_t ilv;               // as EncArgs::ilv (tokens and plaintexts), well-formed uniform tokens only
    unsigned long long *clk;    // as EncArgs::clk
};

// Ratchet trials (Identity.py:865-878): pairs j in [pair_off[t],
// pair_off[t+1]) try key pair_key[j] on token t; first[t] = the rank of the
// first pair whose HMAC verifies over a well-formed token, or 0xFFFFFFFF.
struct TrialArgs {
    const uint32_t *rec;
    const uint8_t *tok;
    const uint64_t *tok_off;
    const uint32_t *tok_len;
    const uint32_t *pair_off;   // n_tok + 1 entries, pair_off[0] = 0, pair_off[n_tok] = n_pairs
    const uint32_t *pair_key;
    uint32_t *first;
    uint32_t n_tok, n_pairs;
};
hipError_t launch_verify_trials(const TrialArgs &a, hipStream_t s);

// HKDF-SHA256 over n items (hkdf_kernels.hip): item i reads ikm + i*ikm_stride
// and salt + i*salt_stride (salt null or salt_len 0: zero key), shares the
// context, writes `length` bytes at out + i*out_stride.
struct HkdfArgs {
    const uint8_t *ikm;
    uint64_t ikm_stride;
    uint32_t ikm_len;
    const uint8_t *salt;
    uint64_t salt_stride;
    uint32_t salt_len;
    const uint8_t *context;
    uint32_t context_len;
    uint8_t *out;
    uint64_t out_stride;
    uint32_t length;
    uint32_t n;
};

// Resource map hashes (resource_kernels.hip): part j = data + part_off[j]
// (part_len[j] bytes), or with part_off null the uniform segmentation
// data[j*sdu, min((j+1)*sdu, size)); salt = salts + part_res[j]*salt_len.
struct MapArgs {
    const uint8_t *data;
    const uint64_t *part_off;
    const uint32_t *part_len;
    uint64_t size;
    uint32_t sdu;
    const uint8_t *salts;
    uint32_t salt_len;
    const uint32_t *part_res;
    uint32_t n_res;
    uint32_t guard;
    uint8_t *out;                  // 4 bytes per part
    uint32_t *first_collision;     // n_res entries or null
    uint32_t n_parts;
};

// Wire-side neighbours (wire_kernels.hip).
struct IfacArgs {
    const uint8_t *pkt;
    const uint64_t *pkt_off;
    const uint32_t *pkt_len;
    uint8_t *ifac;                 // mask: input (n x ifac_size); unmask: output
    uint32_t ifac_size;
    const uint8_t *ifac_key;
    uint32_t key_len;
    uint8_t *out;
    const uint64_t *out_off;
    int32_t *status;               // unmask only
    uint32_t *out_len;             // unmask only, may be null: unmasked length (0 where status != 0)
    uint32_t n;
};
struct PackArgs {
    const uint8_t *flags, *hops, *context;
    const uint8_t *destination_hash;   // 16 B per packet
    const uint8_t *transport_id;       // 16 B per packet or null (HEADER_1)
    uint8_t *out;
    const uint64_t *out_off;
    uint32_t n;
};
uint64_t hdlc_frame_workspace_bytes(uint32_t n);
uint64_t hdlc_deframe_workspace_bytes(uint64_t len);
hipError_t launch_hdlc_frame(const uint8_t *pkt, const uint64_t *off, const uint32_t *len, uint32_t n, uint8_t *out,
                             uint64_t *frame_off, void *ws, hipStream_t s);
hipError_t launch_hdlc_deframe(const uint8_t *buf, uint64_t len, uint32_t hw_mtu, uint32_t ifac_size, uint8_t *out,
                               uint64_t *frame_off, uint32_t *frame_len, int32_t *status, uint64_t *counts,
                               uint64_t max_pairs, void *ws, hipStream_t s, uint32_t line_phase = 0xFFFFFFFFu);
hipError_t launch_ifac(const IfacArgs &a, bool mask, hipStream_t s);
uint64_t frames_compact_workspace_bytes(uint64_t max_pairs);
hipError_t launch_frames_compact(const uint64_t *d_off, const uint32_t *d_len, const int32_t *st,
                                 const uint64_t *counts, uint64_t max_pairs, uint64_t *f_off, uint32_t *f_len,
                                 int64_t *frame_pair, int64_t *n_frames, void *ws, hipStream_t s);
hipError_t launch_token_spans(const void *fields, const uint64_t *pkt_off, uint32_t n, uint64_t *tok_off,
                              uint32_t *tok_len, hipStream_t s);
hipError_t launch_unpack(const uint8_t *pkt, const uint64_t *off, const uint32_t *len, void *fields, uint32_t n,
                         hipStream_t s);
hipError_t launch_pack_headers(const PackArgs &a, hipStream_t s);

hipError_t configure_kernels();

// bytes from device memory `src` to pinned host memory, as GPU stores into the
// mapped host buffer (dst_dev: its device-side address) on stream s
// (copy_kernels.hip; faster than the copy engine's D2H, see there).
// dev_bytes (device pointer, optional): copy min(bytes, *dev_bytes) bytes.
hipError_t launch_store_host(uint8_t *dst_dev, const uint8_t *src, uint64_t bytes, hipStream_t s,
                             const uint64_t *dev_bytes = nullptr);

// Length bucketing: order[] = packet indices grouped by descending AES quad
// count, so that the lanes of a wave carry similar lengths.  `dec` selects
// token lengths (quads of the ciphertext body) instead of plaintext lengths.
// *queue receives a zeroed chunk counter: the token kernels' waves then take
// the ordered packets 64 at a time, longest first (dynamic balance).
constexpr uint32_t SORT_BUCKETS = 4096;
uint64_t sort_workspace_bytes(uint32_t n);    // order[n] + 2 x SORT_BUCKETS counters
hipError_t launch_length_order(const uint32_t *len, uint32_t n, int dec, void *workspace, const uint32_t **order,
                               uint32_t **queue, int n_cu, hipStream_t s);
// Chunk counters for ragged uniform batches (the static stride would leave a
// ragged last pass).  acquire() hands out a 4-byte device counter (and its
// slot number) that no other launch can still be reading once work queued on
// `s` after this call runs (the C-ABI orders slot reuse with an event per
// slot), or null; release(s, slot) is called once after the launch that used
// it has been enqueued on `s`.  Thread-safe, no lock held in between.
struct SpareQueue {
    virtual uint32_t *acquire(hipStream_t s, uint32_t *slot) = 0;
    virtual void release(hipStream_t s, uint32_t slot) = 0;
    virtual ~SpareQueue() {}
};
// Which kernel a batch runs on (RT_KERNEL_*, include/rnstok.h): the routing
// launch_encrypt / launch_decrypt apply, exposed as rt_plan_uniform.
int plan_encrypt(uint32_t n, bool packed, uint32_t uni_len, bool per_key, int n_cu);
int plan_decrypt(uint32_t n, bool packed, uint32_t uni_len, bool per_key, int n_cu);
hipError_t launch_encrypt(const EncArgs &a, int nr, int n_cu, SpareQueue *spare, hipStream_t s);
hipError_t launch_decrypt(const DecArgs &a, int nr, int n_cu, SpareQueue *spare, hipStream_t s);
// Token.verify_hmac (Token.py:77-84) over n tokens: status[i] = 0 (tag
// valid), 1 (len <= 32) or 2 (tag mismatch); no AES, no plaintext.
struct VerifyArgs {
    const uint32_t *rec;
    const uint8_t *tok;
    const uint64_t *tok_off;    // null -> i * tok_stride
    uint64_t tok_stride;
    const uint32_t *tok_len;    // null -> uni_len
    uint32_t uni_len;
    const uint32_t *key_idx;    // null -> key 0
    int32_t *status;
    uint32_t n;
};
hipError_t launch_verify(const VerifyArgs &a, hipStream_t s);
hipError_t launch_map_hashes(const MapArgs &m, hipStream_t s);
hipError_t launch_hkdf(const HkdfArgs &a, hipStream_t s);
hipError_t launch_key_setup(const uint8_t *keys, uint32_t key_len, uint32_t n_keys, const uint8_t *sbox,
                            uint32_t *rec, hipStream_t s);
// HKDF (a.length = key_len, a.out unused) and key setup in one launch: key i
// of the records is Token(hkdf(key_len, ikm_i, salt_i, context)) and the
// derived key never reaches HBM.  Returns hipErrorNotSupported for shapes
// outside the fused kernel's (the caller then runs launch_hkdf +
// launch_key_setup through a temporary).
hipError_t launch_hkdf_key_setup(const HkdfArgs &a, const uint8_t *sbox, uint32_t *rec, int n_cu, hipStream_t s);

}  // namespace rnstok
