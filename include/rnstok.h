/*
 * rnstok.h — C-ABI of the MI355X encrypted-token engine (librnstok.so).
 *
 * Drop-in boundary for Reticulum's per-packet token path.  The reference is
 * pure Python; the maintainer-side binding is a ctypes stub
 * behind the unchanged class surface of RNS/Cryptography/Token.py.  Each
 * entry point names the reference interface it replaces (markqvist/Reticulum
 * 1.4.2, paths relative to the repository root):
 *
 *   rt_keyset_create   Token.__init__            RNS/Cryptography/Token.py:58-74
 *                      (+ the per-call key schedule AES.py:83,100 and the
 *                       per-call HMAC key pad HMAC.py:73-82, hoisted per key)
 *   rt_encrypt*        Token.encrypt             RNS/Cryptography/Token.py:87-97
 *   rt_decrypt*        Token.verify_hmac+decrypt RNS/Cryptography/Token.py:77-84,100-114
 *   rt_verify*         Token.verify_hmac         RNS/Cryptography/Token.py:77-84 (no AES)
 *   rt_token_len       token size arithmetic     Token.py:50 (TOKEN_OVERHEAD) + PKCS7.py:35-39
 *   rt_hkdf*           RNS.Cryptography.hkdf     RNS/Cryptography/HKDF.py:35-62
 *   rt_map_hashes /    Resource hashmap          RNS/Resource.py:426-468 (map hashes + the
 *   rt_resource_hashmap_host                      collision guard), get_map_hash :505-506,
 *                                                receive_part :865-866
 *   rt_hdlc_frame      HDLC.escape + framing     RNS/Interfaces/TCPInterface.py:44-53, :323
 *   rt_hdlc_deframe    HDLC read loop            RNS/Interfaces/TCPInterface.py:387-410, :336-339
 *   rt_hdlc_deframe_slots  the same, each frame in a 128-B-aligned slot
 *   rt_ifac_mask       IFAC on transmit          RNS/Transport.py:1069-1101
 *   rt_ifac_unmask     IFAC on inbound           RNS/Transport.py:1441-1475
 *   rt_packet_unpack   Packet.unpack + get_hash  RNS/Packet.py:236-268, 342-353
 *   rt_packet_pack_headers  Packet.pack header   RNS/Packet.py:167-228
 *   rt_frames_compact  frames a read hands on    RNS/Interfaces/TCPInterface.py:391-401
 *                      (one process_incoming call per frame, in stream order)
 *   rt_token_spans     packet.data (the token)   RNS/Packet.py:262-275 (data after the header)
 *   rt_keyset_create_hkdf  per-packet keying     Identity.py:837-846 (hkdf -> Token(derived_key)),
 *                                                Link.py handshake key derivation
 *   rt_verify_trials*  ratchet trial loop        Identity.py:865-878 (first ratchet whose key
 *                                                opens the token; Token.py:77-84,114)
 *
 * Conventions
 *  - No exceptions cross the boundary.  API misuse returns a negative RT_E_*
 *    code and sets a thread-local message (rt_last_error).  Per-packet
 *    outcomes of decrypt are reported in an int32 status array (RT_ST_*),
 *    mirroring the reference's exception classes (Token.py:78,102,114;
 *    PKCS7.py:45-46): the Python layer maps non-zero status to ValueError.
 *  - The caller owns every buffer; the library never frees caller memory.
 *    rt_encrypt / rt_decrypt take DEVICE pointers and a hipStream_t (as
 *    void*; NULL = HIP's null stream, which is also torch's default stream)
 *    and only enqueue work.
 *    rt_*_host take HOST pointers, stage through the context's workspace and
 *    return after the results are back in host memory.
 *  - Token layout (Token.py:96-97): iv(16) || AES-CBC(ek, iv, PKCS7(pt)) ||
 *    HMAC-SHA256(sk, iv||ct)(32), so len(token) = 16 + 16*(L/16 + 1) + 32.
 *  - Key layout (Token.py:61-70): 64-byte keys -> sk = key[0:32],
 *    ek = key[32:64], AES-256-CBC; 32-byte keys -> sk = key[0:16],
 *    ek = key[16:32], AES-128-CBC.  One keyset holds keys of one length.
 *  - IVs are supplied by the caller (16 bytes per packet), drawn from
 *    os.urandom as in Token.py:89; the library never generates IVs.
 *  - Thread safety: a context may be used from several host threads.  Host
 *    staging calls run on one of the context's staging lanes (each its own
 *    stream, workspace and pinned buffer), so up to 4 run concurrently.
 *    Device calls are re-entrant given distinct output buffers, from any
 *    thread and on any streams.
 *  - Stream ordering of key sets: a key set is built on the stream it was
 *    created on (rt_keyset_create: a staging lane's stream), and every later
 *    launch that reads it, on any stream, first waits for that build.
 *    rt_keyset_destroy never blocks: the records are released once the last
 *    launch on every stream that used them has completed.
 */
#ifndef RNSTOK_H
#define RNSTOK_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RNSTOK_ABI_VERSION 2   /* 2: rt_hdlc_deframe_slots, rt_clock_stamps */

/* Return codes (< 0: API misuse or runtime failure). */
#define RT_OK        0
#define RT_E_INVAL  -1   /* bad argument (NULL pointer, bad key length, ...) */
#define RT_E_HIP    -2   /* HIP runtime error (message in rt_last_error)     */
#define RT_E_NOMEM  -3   /* device or pinned allocation failed               */
#define RT_E_NODEV  -4   /* no usable gfx950 device                          */

/* Per-packet decrypt status. */
#define RT_ST_OK          0  /* plaintext written, pt_len set                    */
#define RT_ST_TOO_SHORT   1  /* len(token) <= 32            (Token.py:78)        */
#define RT_ST_BAD_HMAC    2  /* tag mismatch                (Token.py:102)       */
#define RT_ST_BAD_CT_LEN  3  /* valid tag, ct empty or %16  (Token.py:114 wrap)  */
#define RT_ST_BAD_PAD     4  /* valid tag, last byte > 16   (PKCS7.py:45-46)     */

typedef struct rt_ctx rt_ctx;
typedef struct rt_keyset rt_keyset;

/* ---- library / context --------------------------------------------------- */
int         rt_abi_version(void);
const char *rt_last_error(void);
int         rt_device_count(void);
/* One context per device.  Builds the S-box tables on the device. */
rt_ctx     *rt_create(int device);
void        rt_destroy(rt_ctx *ctx);
/* Number of compute units the context launches over (persistent grid). */
int         rt_num_cus(const rt_ctx *ctx);

/* ---- keys (Token.__init__, Token.py:58-74) ------------------------------- */
/* keys: HOST pointer, n_keys x key_len bytes, key_len 64 (AES-256) or 32
 * (AES-128).  Runs the key-setup kernel: AES encryption and equivalent
 * decryption schedules plus HMAC-SHA256 ipad/opad midstates per key. */
rt_keyset  *rt_keyset_create(rt_ctx *ctx, const uint8_t *keys, uint32_t key_len, uint32_t n_keys);
/* Same, with the raw keys already in DEVICE memory (on-device key tables). */
rt_keyset  *rt_keyset_create_device(rt_ctx *ctx, const uint8_t *d_keys, uint32_t key_len, uint32_t n_keys,
                                    void *stream);
void        rt_keyset_destroy(rt_keyset *ks);
uint32_t    rt_keyset_size(const rt_keyset *ks);

/* ---- sizes --------------------------------------------------------------- */
uint64_t    rt_token_len(uint64_t pt_len);      /* 16 + 16*(pt_len/16+1) + 32 */

/* ---- unit-interleaved device batches (no reference counterpart) ---------- */
/* For batches that are produced and consumed on the device (e.g. the
 * deframer's output feeding decrypt), a layout in which every wave load and
 * store instruction covers 1 KiB of contiguous HBM: 16-B unit u of packet p
 * at buf + 16*(u*n + p).  Plaintexts hold ceil(pt_len/16) units (the last
 * one partial: only its first pt_len % 16 bytes are read), tokens
 * rt_token_len(pt_len)/16 units (IV, ciphertext blocks, 2 tag units), the
 * decrypted plaintext (tok_len - 48)/16 units (pad block included, as
 * rt_decrypt_uniform).  iv: n x 16 B.  Outputs, statuses and error order are
 * those of rt_encrypt_uniform / rt_decrypt_uniform on the same packets;
 * decrypt takes well-formed token lengths only (48 + 16*k, k >= 1), others
 * are RT_E_INVAL.  Always the one-packet-per-lane kernels. */
int rt_encrypt_interleaved(const rt_keyset *ks, const uint8_t *pt, uint32_t pt_len, const uint32_t *key_idx,
                           const uint8_t *iv, uint8_t *tok, uint32_t n, void *stream);
int rt_decrypt_interleaved(const rt_keyset *ks, const uint8_t *tok, uint32_t tok_len, const uint32_t *key_idx,
                           uint8_t *pt, uint32_t *pt_len, int32_t *status, uint32_t n, void *stream);

/* ---- kernel plan (diagnostic; no reference counterpart) ------------------ */
/* The kernel rt_encrypt_uniform (decrypt = 0, len = plaintext bytes) or
 * rt_decrypt_uniform (decrypt = 1, len = token bytes) runs for n packets on
 * ctx's device, with one key (per_packet_keys = 0) or a key_idx array.  Lets
 * tests and callers check which path a batch shape takes (e.g. that the
 * 8-GPU c4 per-rank shard runs the long-token kernels). */
enum {
    RT_KERNEL_GENERAL = 0,      /* one packet per lane (k_encrypt / k_decrypt) */
    RT_KERNEL_ENC_LONG4 = 1,    /* single key, a lane quad per CBC chain (k_encrypt_long4) */
    RT_KERNEL_ENC_LONG = 2,     /* per-packet keys, hashing on waves of their own (k_encrypt_long) */
    RT_KERNEL_DEC_LONG2 = 3,    /* single key, producer/consumer HMAC chains (k_decrypt_long2) */
    RT_KERNEL_ENC_SPLIT = 4     /* single key, AES and HMAC chains on waves of their own (k_encrypt_split) */
};
int         rt_plan_uniform(const rt_ctx *ctx, uint32_t n, uint32_t len, int per_packet_keys, int decrypt);

/* ---- device-resident batch (Token.encrypt over n packets) ---------------- */
/* pt + pt_off[i] holds pt_len[i] plaintext bytes; key_idx[i] selects the key
 * (NULL: key 0 for every packet); iv + 16*i is packet i's IV; the token is
 * written at tok + tok_off[i] (rt_token_len(pt_len[i]) bytes).  Offsets need
 * no alignment.  All pointers are device pointers. */
int rt_encrypt(const rt_keyset *ks, const uint8_t *pt, const uint64_t *pt_off, const uint32_t *pt_len,
               const uint32_t *key_idx, const uint8_t *iv, uint8_t *tok, const uint64_t *tok_off,
               uint32_t n, void *stream);
/* Fixed-length batch: packet i at pt + i*pt_stride (pt_len bytes), token at
 * tok + i*tok_stride.  pt may be null when pt_len is 0. */
int rt_encrypt_uniform(const rt_keyset *ks, const uint8_t *pt, uint64_t pt_stride, uint32_t pt_len,
                       const uint32_t *key_idx, const uint8_t *iv, uint8_t *tok, uint64_t tok_stride,
                       uint32_t n, void *stream);

/* ---- device-resident batch (Token.decrypt over n tokens) ----------------- */
/* tok + tok_off[i] holds tok_len[i] token bytes; plaintext (up to
 * tok_len[i]-48 bytes, including the pad block) is written at pt + pt_off[i];
 * pt_len[i] receives the unpadded length on RT_ST_OK, the offending pad
 * byte on RT_ST_BAD_PAD (authenticated data), 0 otherwise; status[i] one
 * of RT_ST_*.  On any non-OK status the packet's plaintext region is zeroed
 * (unauthenticated plaintext is never left behind). */
int rt_decrypt(const rt_keyset *ks, const uint8_t *tok, const uint64_t *tok_off, const uint32_t *tok_len,
               const uint32_t *key_idx, uint8_t *pt, const uint64_t *pt_off, uint32_t *pt_len,
               int32_t *status, uint32_t n, void *stream);
int rt_decrypt_uniform(const rt_keyset *ks, const uint8_t *tok, uint64_t tok_stride, uint32_t tok_len,
                       const uint32_t *key_idx, uint8_t *pt, uint64_t pt_stride, uint32_t *pt_len,
                       int32_t *status, uint32_t n, void *stream);

/* ---- device-resident batch (Token.verify_hmac over n tokens) ------------- */
/* status[i] = RT_ST_OK when token i's last 32 bytes equal HMAC-SHA256(sk,
 * token[:-32]), RT_ST_BAD_HMAC when they do not, RT_ST_TOO_SHORT when
 * tok_len[i] <= 32 (Token.py:77-84: any length above 32 is hashed, whole AES
 * blocks or not).  Runs no AES and writes nothing but the status.  DEVICE
 * pointers; rt_verify_host takes HOST pointers and returns when `status` is
 * filled. */
int rt_verify(const rt_keyset *ks, const uint8_t *tok, const uint64_t *tok_off, const uint32_t *tok_len,
              const uint32_t *key_idx, int32_t *status, uint32_t n, void *stream);
int rt_verify_host(const rt_keyset *ks, const uint8_t *tok, const uint64_t *tok_off, const uint32_t *tok_len,
                   const uint32_t *key_idx, int32_t *status, uint32_t n);

/* ---- irregular batches: length bucketing -------------------------------- */
/* With RT_F_SORT_BY_LENGTH the batch is first grouped by length on the device
 * (three small kernels on the same stream) so that the lanes of a wavefront
 * carry packets of similar length; outputs stay at their own offsets, so the
 * result is identical to rt_encrypt / rt_decrypt.  `workspace` is a DEVICE
 * buffer of at least rt_workspace_bytes(n) bytes, owned by the caller and not
 * reused until the call's work on `stream` has completed. */
#define RT_F_SORT_BY_LENGTH 1u
uint64_t rt_workspace_bytes(uint32_t n);
int rt_encrypt_ex(const rt_keyset *ks, const uint8_t *pt, const uint64_t *pt_off, const uint32_t *pt_len,
                  const uint32_t *key_idx, const uint8_t *iv, uint8_t *tok, const uint64_t *tok_off,
                  uint32_t n, uint32_t flags, void *workspace, void *stream);
int rt_decrypt_ex(const rt_keyset *ks, const uint8_t *tok, const uint64_t *tok_off, const uint32_t *tok_len,
                  const uint32_t *key_idx, uint8_t *pt, const uint64_t *pt_off, uint32_t *pt_len,
                  int32_t *status, uint32_t n, uint32_t flags, void *workspace, void *stream);

/* ---- host-buffer convenience (PCIe-inclusive path) ----------------------- */
/* Same meaning with HOST pointers; H2D, kernel, D2H on a staging lane's
 * stream, synchronised (that stream only) before return. */
int rt_encrypt_host(const rt_keyset *ks, const uint8_t *pt, const uint64_t *pt_off, const uint32_t *pt_len,
                    const uint32_t *key_idx, const uint8_t *iv, uint8_t *tok, const uint64_t *tok_off,
                    uint32_t n);
int rt_decrypt_host(const rt_keyset *ks, const uint8_t *tok, const uint64_t *tok_off, const uint32_t *tok_len,
                    const uint32_t *key_idx, uint8_t *pt, const uint64_t *pt_off, uint32_t *pt_len,
                    int32_t *status, uint32_t n);

/* ---- key derivation (RNS.Cryptography.hkdf, HKDF.py:35-62) -------------- */
/* n independent HKDF-SHA256 derivations.  Item i: input key material
 * ikm + i*ikm_stride (ikm_len bytes; 0 is allowed, as b"" is in the
 * reference), salt + i*salt_stride (salt_len bytes; salt NULL or salt_len 0
 * means the reference's default of 32 zero bytes, HKDF.py:45-46; salts over
 * 64 bytes are hashed first as HMAC.py does with long keys; salt_stride 0
 * shares one salt row across all items, as Identity.encrypt does for packets
 * to one identity, and the salt's HMAC midstates are then computed once per
 * lane rather than once per item), a context shared
 * by all items (NULL / 0: empty, HKDF.py:48-49); `length` >= 1 output bytes
 * are written at out + i*out_stride (length 0 is RT_E_INVAL, HKDF.py:40-41).
 * Output blocks past 255 wrap the counter byte exactly as HKDF.py:60 does.
 * rt_hkdf takes DEVICE pointers and only enqueues; rt_hkdf_host takes HOST
 * pointers and returns when `out` is filled. */
int rt_hkdf(rt_ctx *ctx, const uint8_t *ikm, uint64_t ikm_stride, uint32_t ikm_len,
            const uint8_t *salt, uint64_t salt_stride, uint32_t salt_len,
            const uint8_t *context, uint32_t context_len,
            uint8_t *out, uint64_t out_stride, uint32_t length, uint32_t n, void *stream);
int rt_hkdf_host(rt_ctx *ctx, const uint8_t *ikm, uint64_t ikm_stride, uint32_t ikm_len,
                 const uint8_t *salt, uint64_t salt_stride, uint32_t salt_len,
                 const uint8_t *context, uint32_t context_len,
                 uint8_t *out, uint64_t out_stride, uint32_t length, uint32_t n);
/* Per-packet keying: derive n token keys of key_len (64 or 32) bytes with
 * HKDF (arguments as rt_hkdf, DEVICE pointers) and build their key tables,
 * without the derived keys ever leaving the device: key i of the keyset is
 * Token(hkdf(key_len, ikm_i, salt_i, context)) as Identity.encrypt /
 * __decrypt construct it (Identity.py:837-846).  Encrypt with key_idx[i] = i. */
rt_keyset *rt_keyset_create_hkdf(rt_ctx *ctx, const uint8_t *ikm, uint64_t ikm_stride, uint32_t ikm_len,
                                 const uint8_t *salt, uint64_t salt_stride, uint32_t salt_len,
                                 const uint8_t *context, uint32_t context_len, uint32_t key_len, uint32_t n,
                                 void *stream);

/* ---- ratchet trials (Identity.decrypt, RNS/Identity.py:865-878) --------- */
/* Identity.decrypt tries the receiver's ratchets in order and keeps the first
 * whose derived token key opens the token.  Token t has the candidate keys
 * pair_key[pair_off[t] .. pair_off[t+1]) of the key set, in the caller's
 * ratchet order (pair_off: n_tok + 1 entries from 0 to n_pairs).  first[t]
 * receives the rank (0-based, within token t's candidates) of the first
 * candidate whose HMAC-SHA256 tag verifies over a well-formed token
 * (len >= 64, len - 48 a multiple of 16; Token.py:77-84,114), or 0xFFFFFFFF.
 * Decrypting each opened token with that key (rt_decrypt* with key_idx)
 * completes the loop: a BAD_PAD there means no ratchet opens it, as every
 * later candidate that verifies is the same key.  rt_verify_trials takes
 * DEVICE pointers and only enqueues; _host takes HOST pointers, validates
 * the CSR and key indices, and returns when `first` is filled. */
int rt_verify_trials(const rt_keyset *ks, const uint8_t *tok, const uint64_t *tok_off, const uint32_t *tok_len,
                     const uint32_t *pair_off, const uint32_t *pair_key, uint32_t *first, uint32_t n_tok,
                     uint32_t n_pairs, void *stream);
int rt_verify_trials_host(const rt_keyset *ks, const uint8_t *tok, const uint64_t *tok_off, const uint32_t *tok_len,
                          const uint32_t *pair_off, const uint32_t *pair_key, uint32_t *first, uint32_t n_tok,
                          uint32_t n_pairs);

/* ---- Resource hashmap (RNS/Resource.py:426-468, 505-506) ---------------- */
/* map_hash_j = SHA-256(part_j || salt)[:4] for n_parts parts, DEVICE pointers.
 * Part j is data + part_off[j] (part_len[j] bytes) when part_off/part_len are
 * given, else the uniform segmentation of one resource that the sender uses:
 * data[j*sdu, min((j+1)*sdu, size)) with n_parts = ceil(size / sdu).  The
 * salt is the resource's random_hash (RANDOM_HASH_SIZE = 4 bytes): salts +
 * part_res[j]*salt_len (part_res NULL: every part uses salts[0..salt_len)).
 * map_hashes receives 4 bytes per part (MAPHASH_LEN).  If first_collision is
 * not NULL it receives, per resource, the first (batch-wide) part index whose map hash
 * equals one of the previous `guard` map hashes of the same resource
 * (ResourceAdvertisement.COLLISION_GUARD_SIZE = 224 in the reference), or
 * 0xFFFFFFFF: the point where the reference's loop breaks to draw a new
 * random_hash.  Parts of one resource must be contiguous and in order. */
int rt_map_hashes(rt_ctx *ctx, const uint8_t *data, const uint64_t *part_off, const uint32_t *part_len,
                  uint64_t size, uint32_t sdu, const uint8_t *salts, uint32_t salt_len, const uint32_t *part_res,
                  uint32_t n_res, uint32_t guard, uint8_t *map_hashes, uint32_t *first_collision, uint32_t n_parts,
                  void *stream);
/* One resource in HOST memory (uniform segmentation); returns when the
 * hashmap (4*ceil(size/sdu) bytes) and *first_collision are written. */
int rt_resource_hashmap_host(rt_ctx *ctx, const uint8_t *data, uint64_t size, uint32_t sdu,
                             const uint8_t *random_hash, uint32_t rh_len, uint32_t guard, uint8_t *hashmap,
                             uint32_t *first_collision);

/* ---- wire-side neighbours (framing, IFAC, packet header) --------------- */
/* HDLC framing of n packets into one stream, in order: frame i is
 * 7E || escape(packet i) || 7E (escape: 7D -> 7D 5D, 7E -> 7D 5E) at
 * out + frame_off[i]; frame_off has n+1 entries, frame_off[n] = total bytes.
 * out needs at most sum(2*len+2) bytes.  DEVICE pointers; `workspace` of
 * rt_hdlc_frame_workspace_bytes(n) bytes. */
uint64_t rt_hdlc_frame_workspace_bytes(uint32_t n);
int rt_hdlc_frame(rt_ctx *ctx, const uint8_t *pkt, const uint64_t *pkt_off, const uint32_t *pkt_len, uint32_t n,
                  uint8_t *out, uint64_t *frame_off, void *workspace, void *stream);
/* One pass of the HDLC read loop over buf[0, len) (everything received so
 * far).  For every pair of consecutive 7E flags k, k+1 (at most max_pairs):
 * the frame between them, unescaped with the loop's two replace passes, is
 * written at out + frame_off[k] (its position in buf, so `out` needs len
 * bytes), frame_len[k] bytes, and status[k] is RT_FRAME_OK (handed to
 * process_incoming), RT_FRAME_BAD_LEN (dropped by check_frame_len: length <=
 * HEADER_MINSIZE = 19 or > hw_mtu + ifac_size) or RT_FRAME_EMPTY (skipped).
 * counts[0] = number of pairs, counts[1] = bytes consumed: the loop keeps
 * buf[counts[1], len) for the next read (all of it is dropped when no flag is
 * present or the tail from the last flag exceeds 2*hw_mtu).  DEVICE
 * pointers; `workspace` of rt_hdlc_deframe_workspace_bytes(len) bytes. */
#define RT_FRAME_OK      0
#define RT_FRAME_BAD_LEN 1
#define RT_FRAME_EMPTY   2
uint64_t rt_hdlc_deframe_workspace_bytes(uint64_t len);
int rt_hdlc_deframe(rt_ctx *ctx, const uint8_t *buf, uint64_t len, uint32_t hw_mtu, uint32_t ifac_size, uint8_t *out,
                    uint64_t *frame_off, uint32_t *frame_len, int32_t *status, uint64_t *counts, uint64_t max_pairs,
                    void *workspace, void *stream);
/* rt_hdlc_deframe with every frame in its own 128-B-aligned slot instead of
 * at its position in buf: frame k is written at the first offset >=
 * pos_k + 1 + 128*k (pos_k: its opening flag) at which byte line_phase (< 128)
 * of the frame starts a 128-B line of memory, so `out` needs
 * len + 128 * (max_pairs + 1) bytes.  Frame bytes, lengths, statuses and
 * counts are those of rt_hdlc_deframe; only frame_off differs.  With
 * line_phase = 35 a HEADER_1 packet at the frame's offset (as it is, or
 * IFAC-unmasked into another buffer at the same offset) has its token
 * ciphertext on a line. */
int rt_hdlc_deframe_slots(rt_ctx *ctx, const uint8_t *buf, uint64_t len, uint32_t hw_mtu, uint32_t ifac_size,
                          uint32_t line_phase, uint8_t *out, uint64_t *frame_off, uint32_t *frame_len, int32_t *status,
                          uint64_t *counts, uint64_t max_pairs, void *workspace, void *stream);
/* The frames one rt_hdlc_deframe pass hands on (pair k < counts[0] with
 * status[k] == RT_FRAME_OK), in stream order, to the front of f_off / f_len
 * (their offsets and lengths in the deframed buffer) and frame_pair (k);
 * *n_frames (device int64) = their number.  Entries n_frames .. max_pairs-1
 * are f_off 0, f_len 0, frame_pair -1, so per-packet stages can run over all
 * max_pairs entries without the host learning n_frames.  The outputs must not
 * overlap frame_off / frame_len (compaction in place would race; RT_E_INVAL).
 * DEVICE pointers; `workspace` of rt_frames_compact_workspace_bytes(max_pairs)
 * bytes. */
uint64_t rt_frames_compact_workspace_bytes(uint64_t max_pairs);
int rt_frames_compact(rt_ctx *ctx, const uint64_t *frame_off, const uint32_t *frame_len, const int32_t *status,
                      const uint64_t *counts, uint64_t max_pairs, uint64_t *f_off, uint32_t *f_len,
                      int64_t *frame_pair, int64_t *n_frames, void *workspace, void *stream);
/* IFAC on transmit: packet i (pkt + pkt_off[i], pkt_len[i] >= 2 bytes) with
 * its access code ifac + i*ifac_size (the last ifac_size bytes of the
 * interface identity's Ed25519 signature of the packet, computed by the
 * caller; signing stays on the host) becomes pkt_len[i] + ifac_size bytes at
 * out + out_off[i]: IFAC flag set, IFAC inserted after the 2 header bytes,
 * all but the IFAC masked with HKDF(len + ifac_size, ifac, ifac_key).
 * ifac_key: key_len (<= 64) bytes shared by the batch.  DEVICE pointers. */
int rt_ifac_mask(rt_ctx *ctx, const uint8_t *pkt, const uint64_t *pkt_off, const uint32_t *pkt_len,
                 const uint8_t *ifac, uint32_t ifac_size, const uint8_t *ifac_key, uint32_t key_len, uint8_t *out,
                 const uint64_t *out_off, uint32_t n, void *stream);
/* IFAC on inbound: status[i] = 0 when the packet carries the IFAC flag and
 * is longer than 2 + ifac_size; then its IFAC goes to ifac_out + i*ifac_size
 * and the unmasked packet without it (pkt_len[i] - ifac_size bytes, flag
 * cleared) to out + out_off[i].  status 1: the reference drops the packet
 * before signing.  out_len (may be NULL) receives the unmasked length,
 * pkt_len[i] - ifac_size, where status[i] is 0 and 0 elsewhere, ready as
 * rt_packet_unpack's pkt_len.  The caller then compares ifac with the tail of
 * sign(unmasked packet) (Transport.py:1477-1481). */
int rt_ifac_unmask(rt_ctx *ctx, const uint8_t *pkt, const uint64_t *pkt_off, const uint32_t *pkt_len,
                   uint32_t ifac_size, const uint8_t *ifac_key, uint32_t key_len, uint8_t *ifac_out, uint8_t *out,
                   const uint64_t *out_off, int32_t *status, uint32_t *out_len, uint32_t n, void *stream);
/* Packet.unpack + get_hash per packet (96 bytes).  ok = 0 where unpack
 * returns False (hop count >= 128, packet too short for its header). */
typedef struct rt_packet_fields {
    uint8_t  ok, flags, hops, header_type, context_flag, transport_type, destination_type, packet_type;
    uint8_t  context, reserved[3];
    uint32_t data_offset, data_len;     /* data = packet[data_offset : data_offset + data_len] */
    uint8_t  transport_id[16];          /* HEADER_2 only */
    uint8_t  destination_hash[16];
    uint8_t  packet_hash[32];           /* SHA-256(flags & 0x0F || packet[2 or 18:]) */
    uint8_t  reserved2[12];
} rt_packet_fields;
int rt_packet_unpack(rt_ctx *ctx, const uint8_t *pkt, const uint64_t *pkt_off, const uint32_t *pkt_len,
                     rt_packet_fields *fields, uint32_t n, void *stream);
/* The token inside each unpacked packet: tok_off[i] = pkt_off[i] +
 * fields[i].data_offset, tok_len[i] = fields[i].data_len where fields[i].ok;
 * tok_off[i] = pkt_off[i], tok_len[i] = 0 (rejected by rt_decrypt as too
 * short) elsewhere.  Feeds rt_decrypt straight from rt_packet_unpack's
 * records.  DEVICE pointers. */
int rt_token_spans(rt_ctx *ctx, const rt_packet_fields *fields, const uint64_t *pkt_off, uint32_t n,
                   uint64_t *tok_off, uint32_t *tok_len, void *stream);
/* Packet.pack's header for n packets at out + out_off[i]: flags, hops (NULL:
 * 0), [transport_id (16 B each; NULL: HEADER_1 for all)], destination hash
 * (16 B each), context — 19 or 35 bytes; the payload (a token from
 * rt_encrypt, written at out_off[i] + header length) follows. */
int rt_packet_pack_headers(rt_ctx *ctx, const uint8_t *flags, const uint8_t *hops, const uint8_t *transport_id,
                           const uint8_t *destination_hash, const uint8_t *context, uint8_t *out,
                           const uint64_t *out_off, uint32_t n, void *stream);

/* ---- memory helpers (so a non-torch host can drive the device API) ------- */
/* rt_memcpy_d2h: a pinned (page-locked, mapped) destination, e.g. from
 * rt_host_alloc, is written by GPU stores into the mapped buffer on `stream`
 * (faster than the copy engine's device-to-host path on MI355X, and it
 * shares the link with a copy-engine H2D); a pageable one is copied with
 * hipMemcpyAsync.  Either way `dst` is valid once `stream` has run. */
void *rt_device_alloc(rt_ctx *ctx, uint64_t bytes);
void  rt_device_free(rt_ctx *ctx, void *p);
void *rt_host_alloc(uint64_t bytes);            /* pinned */
void  rt_host_free(void *p);
int   rt_memcpy_h2d(rt_ctx *ctx, void *dst, const void *src, uint64_t bytes, void *stream);
int   rt_memcpy_d2h(rt_ctx *ctx, void *dst, const void *src, uint64_t bytes, void *stream);
/* rt_memcpy_d2h_upto: min(max_bytes, *d_bytes) bytes, the count read on the
 * device at run time (d_bytes: a DEVICE 64-bit count on the context's GPU,
 * e.g. frame_off[n] of rt_hdlc_frame, a size the host does not know without
 * a sync; read as signed, so zero or negative copies nothing), as GPU stores
 * into a pinned `dst` (RT_E_INVAL for any other destination); bytes of `dst`
 * past the count are not written. */
int   rt_memcpy_d2h_upto(rt_ctx *ctx, void *dst, const void *src, uint64_t max_bytes, const uint64_t *d_bytes,
                         void *stream);
int   rt_stream_sync(rt_ctx *ctx, void *stream);

/* ---- launch clock (measurement; no reference counterpart) ----------------
 * rt_clock_stamps: from the next launch on, every workgroup of the context's
 * encrypt and decrypt kernels (the one-packet-per-lane, split and long-token
 * kernels of rt_encrypt* / rt_decrypt*) adds its span to `acc`, a DEVICE buffer of
 * RT_CLOCK_WORDS uint64 on the context's GPU (null: stop stamping).  Words
 * [4k .. 4k+3], k = RT_CLOCK_ENCRYPT / RT_CLOCK_DECRYPT: the sum of the
 * workgroups' spans in shader clock cycles, the same spans in 100 MHz
 * real-time ticks, the number of workgroups stamped, the number of launches.
 * The run's sustained shader clock is words[0] / words[1] x 100 MHz and the
 * cycles per launch words[0] / words[2] (one persistent workgroup per CU).
 * The caller zeroes `acc` and reads it after the stamped launches complete. */
#define RT_CLOCK_WORDS 8
#define RT_CLOCK_ENCRYPT 0
#define RT_CLOCK_DECRYPT 1
int   rt_clock_stamps(rt_ctx *ctx, uint64_t *acc);

#ifdef __cplusplus
}
#endif
#endif /* RNSTOK_H */
