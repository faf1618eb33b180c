/*
 * A C host on the C-ABI alone (include/rnstok.h; no Python, no torch): the
 * binding a non-Python Reticulum host would write.  Test infrastructure:
 * outputs are checked against the C oracle (oracle/token_oracle.c), which
 * only tests may link.  Run by tests/test_c_host_gpu.py.
 *
 *   1. Token.encrypt / Token.decrypt / Token.verify_hmac over host buffers
 *      (rt_encrypt_host, rt_decrypt_host, rt_verify_host): ragged lengths
 *      0..700 B, two keys, every token equal to the oracle's, tampered tags
 *      rejected (RT_ST_BAD_HMAC).
 *   2. The same batch device-resident (rt_device_alloc, rt_memcpy_h2d,
 *      rt_encrypt, rt_decrypt, rt_memcpy_d2h into pinned and pageable host
 *      memory, rt_stream_sync).
 *   3. The interface path composed on the device with no host sync between
 *      stages: rt_encrypt into packet rows, rt_packet_pack_headers,
 *      rt_ifac_mask, rt_hdlc_frame; then rt_hdlc_deframe, rt_frames_compact,
 *      rt_ifac_unmask (out_len), rt_packet_unpack, rt_token_spans,
 *      rt_decrypt: every plaintext back, every token the oracle's.
 *
 * Exit status 0 and one "ok" line on success; a message and 1 otherwise.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rnstok.h"

/* oracle/token_oracle.c (test infrastructure) */
uint64_t oracle_token_len(uint32_t pt_len);
int64_t oracle_token_encrypt(const uint8_t *key, uint32_t klen, const uint8_t iv[16], const uint8_t *pt, uint32_t L,
                             uint8_t *tok);

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint32_t rnd(void) {
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return (uint32_t)(rng_state >> 11);
}
static void fill(uint8_t *p, uint64_t n) {
    for (uint64_t i = 0; i < n; ++i) p[i] = (uint8_t)rnd();
}

#define CHECK(cond, ...)                                                            \
    do {                                                                            \
        if (!(cond)) {                                                              \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);                    \
            fprintf(stderr, __VA_ARGS__);                                           \
            fprintf(stderr, " (rt_last_error: %s)\n", rt_last_error());             \
            exit(1);                                                                \
        }                                                                           \
    } while (0)
#define RT(call) CHECK((call) == RT_OK, "%s", #call)

static void *dalloc(rt_ctx *c, uint64_t bytes) {
    void *p = rt_device_alloc(c, bytes ? bytes : 1);
    CHECK(p != NULL, "rt_device_alloc(%llu)", (unsigned long long)bytes);
    return p;
}
static void *h2d(rt_ctx *c, const void *src, uint64_t bytes) {
    void *d = dalloc(c, bytes);
    if (bytes) RT(rt_memcpy_h2d(c, d, src, bytes, NULL));
    return d;
}
static void d2h(rt_ctx *c, void *dst, const void *src, uint64_t bytes) {
    if (bytes) RT(rt_memcpy_d2h(c, dst, src, bytes, NULL));
    RT(rt_stream_sync(c, NULL));
}

enum { N = 777, MAXL = 700, NK = 2 };

static void token_batch(rt_ctx *c, rt_keyset *ks, const uint8_t *keys) {
    uint32_t *len = malloc(4 * N), *kidx = malloc(4 * N), *tlen = malloc(4 * N), *olen = malloc(4 * N);
    uint64_t *off = malloc(8 * N), *toff = malloc(8 * N);
    int32_t *st = malloc(4 * N), *vst = malloc(4 * N);
    uint8_t *iv = malloc(16 * N);
    uint64_t pbytes = 0, tbytes = 0;
    for (int i = 0; i < N; ++i) {
        len[i] = i < 3 ? (uint32_t)(16 * i) : rnd() % (MAXL + 1);     /* 0, 16, 32 and ragged */
        kidx[i] = rnd() % NK;
        off[i] = pbytes;
        toff[i] = tbytes;
        tlen[i] = (uint32_t)rt_token_len(len[i]);
        pbytes += len[i];
        tbytes += tlen[i];
    }
    uint8_t *pt = malloc(pbytes + 1), *tok = malloc(tbytes), *ref = malloc(tbytes), *back = malloc(tbytes);
    fill(pt, pbytes);
    fill(iv, 16 * N);
    for (int i = 0; i < N; ++i) {
        int64_t t = oracle_token_encrypt(keys + 64 * kidx[i], 64, iv + 16 * i, pt + off[i], len[i], ref + toff[i]);
        CHECK(t == (int64_t)tlen[i], "oracle token length %d", i);
    }

    /* 1. host buffers */
    RT(rt_encrypt_host(ks, pt, off, len, kidx, iv, tok, toff, N));
    CHECK(memcmp(tok, ref, tbytes) == 0, "rt_encrypt_host tokens differ from the oracle's");
    RT(rt_decrypt_host(ks, tok, toff, tlen, kidx, back, toff, olen, st, N));
    for (int i = 0; i < N; ++i) {
        CHECK(st[i] == RT_ST_OK && olen[i] == len[i], "decrypt status %d len %u (packet %d)", st[i], olen[i], i);
        CHECK(memcmp(back + toff[i], pt + off[i], len[i]) == 0, "plaintext %d", i);
    }
    for (int i = 5; i < N; i += 97) tok[toff[i] + tlen[i] - 1] ^= 1;    /* last tag byte */
    RT(rt_verify_host(ks, tok, toff, tlen, kidx, vst, N));
    RT(rt_decrypt_host(ks, tok, toff, tlen, kidx, back, toff, olen, st, N));
    for (int i = 0; i < N; ++i) {
        const int32_t want = (i >= 5 && (i - 5) % 97 == 0) ? RT_ST_BAD_HMAC : RT_ST_OK;
        CHECK(st[i] == want && vst[i] == want, "tampered batch: packet %d status %d / %d", i, st[i], vst[i]);
    }

    /* 2. device-resident, D2H into pinned (GPU stores) and pageable memory */
    uint8_t *d_pt = h2d(c, pt, pbytes), *d_iv = h2d(c, iv, 16 * N), *d_tok = dalloc(c, tbytes);
    uint64_t *d_off = h2d(c, off, 8 * N), *d_toff = h2d(c, toff, 8 * N);
    uint32_t *d_len = h2d(c, len, 4 * N), *d_tlen = h2d(c, tlen, 4 * N), *d_kidx = h2d(c, kidx, 4 * N);
    uint32_t *d_olen = dalloc(c, 4 * N);
    int32_t *d_st = dalloc(c, 4 * N);
    uint8_t *d_back = dalloc(c, tbytes);
    RT(rt_encrypt(ks, d_pt, d_off, d_len, d_kidx, d_iv, d_tok, d_toff, N, NULL));
    uint8_t *pinned = rt_host_alloc(tbytes);
    CHECK(pinned != NULL, "rt_host_alloc");
    d2h(c, pinned, d_tok, tbytes);
    CHECK(memcmp(pinned, ref, tbytes) == 0, "rt_encrypt tokens (pinned D2H) differ from the oracle's");
    memset(back, 0, tbytes);
    d2h(c, back, d_tok, tbytes);
    CHECK(memcmp(back, ref, tbytes) == 0, "rt_encrypt tokens (pageable D2H) differ from the oracle's");
    RT(rt_decrypt(ks, d_tok, d_toff, d_tlen, d_kidx, d_back, d_toff, d_olen, d_st, N, NULL));
    d2h(c, back, d_back, tbytes);
    d2h(c, st, d_st, 4 * N);
    d2h(c, olen, d_olen, 4 * N);
    for (int i = 0; i < N; ++i)
        CHECK(st[i] == RT_ST_OK && olen[i] == len[i] && memcmp(back + toff[i], pt + off[i], len[i]) == 0,
              "device decrypt packet %d", i);
    rt_host_free(pinned);
    void *dev_bufs[] = {d_pt, d_iv, d_tok, d_off, d_toff, d_len, d_tlen, d_kidx, d_olen, d_st, d_back};
    for (unsigned k = 0; k < sizeof dev_bufs / sizeof dev_bufs[0]; ++k) rt_device_free(c, dev_bufs[k]);
    free(len); free(kidx); free(tlen); free(olen); free(off); free(toff); free(st); free(vst); free(iv);
    free(pt); free(tok); free(ref); free(back);
}

enum { NP = 3001, PL = 383, ISZ = 16, HDR = 19 };

static void interface_path(rt_ctx *c, rt_keyset *ks, const uint8_t *key, int slots) {
    const uint32_t tl = (uint32_t)rt_token_len(PL), rl = HDR + tl, ml = rl + ISZ;
    uint8_t *pt = malloc((uint64_t)NP * PL), *iv = malloc(16 * NP), *dh = malloc(16 * NP), *ctx = malloc(NP);
    uint8_t *ifac = malloc((uint64_t)NP * ISZ), ikey[64];
    uint64_t *roff = malloc(8 * NP), *moff = malloc(8 * NP);
    uint32_t *rlen = malloc(4 * NP), *mlen = malloc(4 * NP);
    fill(pt, (uint64_t)NP * PL); fill(iv, 16 * NP); fill(dh, 16 * NP); fill(ctx, NP);
    fill(ifac, (uint64_t)NP * ISZ); fill(ikey, 64);
    for (int i = 0; i < NP; ++i) {
        roff[i] = (uint64_t)i * rl; rlen[i] = rl;
        moff[i] = (uint64_t)i * ml; mlen[i] = ml;
    }
    uint8_t *zero = calloc(NP, 1);
    /* outbound: tokens straight into the packet rows after the 19-B header */
    uint8_t *d_pt = h2d(c, pt, (uint64_t)NP * PL), *d_iv = h2d(c, iv, 16 * NP), *d_dh = h2d(c, dh, 16 * NP);
    uint8_t *d_ctx = h2d(c, ctx, NP), *d_zero = h2d(c, zero, NP), *d_ifac = h2d(c, ifac, (uint64_t)NP * ISZ);
    uint8_t *d_ikey = h2d(c, ikey, 64), *d_raw = dalloc(c, (uint64_t)NP * rl), *d_mask = dalloc(c, (uint64_t)NP * ml);
    uint64_t *d_roff = h2d(c, roff, 8 * NP), *d_moff = h2d(c, moff, 8 * NP), *d_foff = dalloc(c, 8 * (NP + 1));
    uint32_t *d_rlen = h2d(c, rlen, 4 * NP), *d_mlen = h2d(c, mlen, 4 * NP);
    const uint64_t fcap = (uint64_t)NP * (2 * ml + 2);
    uint8_t *d_framed = dalloc(c, fcap);
    void *d_fws = dalloc(c, rt_hdlc_frame_workspace_bytes(NP));
    RT(rt_encrypt_uniform(ks, d_pt, PL, PL, NULL, d_iv, d_raw + HDR, rl, NP, NULL));
    RT(rt_packet_pack_headers(c, d_zero, d_zero, NULL, d_dh, d_ctx, d_raw, d_roff, NP, NULL));
    RT(rt_ifac_mask(c, d_raw, d_roff, d_rlen, d_ifac, ISZ, d_ikey, 64, d_mask, d_moff, NP, NULL));
    RT(rt_hdlc_frame(c, d_mask, d_moff, d_mlen, NP, d_framed, d_foff, d_fws, NULL));
    uint64_t total = 0;
    d2h(c, &total, d_foff + NP, 8);              /* the stream's length: what a socket write needs */
    CHECK(total > (uint64_t)NP * (ml + 2) && total <= fcap, "framed length %llu", (unsigned long long)total);

    /* inbound: one read of that stream, no host sync until the plaintexts;
     * with slots, every frame in its own 128-B-aligned slot (token ciphertext
     * of the unmasked packet on a line) */
    const uint64_t mp = 2 * NP, cap = slots ? total + 128 * (mp + 1) : total;
    uint8_t *d_out = dalloc(c, cap), *d_un = dalloc(c, cap), *d_ptb = dalloc(c, cap);
    uint8_t *d_ifo = dalloc(c, mp * ISZ);
    uint64_t *d_doff = dalloc(c, 8 * mp), *d_counts = dalloc(c, 16), *d_coff = dalloc(c, 8 * mp);
    uint64_t *d_toff = dalloc(c, 8 * mp);
    uint32_t *d_dlen = dalloc(c, 4 * mp), *d_clen = dalloc(c, 4 * mp), *d_plen = dalloc(c, 4 * mp);
    uint32_t *d_tlen = dalloc(c, 4 * mp), *d_olen = dalloc(c, 4 * mp);
    int32_t *d_dst = dalloc(c, 4 * mp), *d_ist = dalloc(c, 4 * mp), *d_st = dalloc(c, 4 * mp);
    int64_t *d_pair = dalloc(c, 8 * mp), *d_nf = dalloc(c, 8);
    rt_packet_fields *d_fields = dalloc(c, sizeof(rt_packet_fields) * mp);
    void *d_dws = dalloc(c, rt_hdlc_deframe_workspace_bytes(total));
    void *d_cws = dalloc(c, rt_frames_compact_workspace_bytes(mp));
    if (slots)
        RT(rt_hdlc_deframe_slots(c, d_framed, total, 262144, ISZ, HDR + 16, d_out, d_doff, d_dlen, d_dst, d_counts, mp,
                                 d_dws, NULL));
    else
        RT(rt_hdlc_deframe(c, d_framed, total, 262144, ISZ, d_out, d_doff, d_dlen, d_dst, d_counts, mp, d_dws, NULL));
    RT(rt_frames_compact(c, d_doff, d_dlen, d_dst, d_counts, mp, d_coff, d_clen, d_pair, d_nf, d_cws, NULL));
    RT(rt_ifac_unmask(c, d_out, d_coff, d_clen, ISZ, d_ikey, 64, d_ifo, d_un, d_coff, d_ist, d_plen, (uint32_t)mp,
                      NULL));
    RT(rt_packet_unpack(c, d_un, d_coff, d_plen, d_fields, (uint32_t)mp, NULL));
    RT(rt_token_spans(c, d_fields, d_coff, (uint32_t)mp, d_toff, d_tlen, NULL));
    RT(rt_decrypt(ks, d_un, d_toff, d_tlen, NULL, d_ptb, d_toff, d_olen, d_st, (uint32_t)mp, NULL));

    int64_t nf = 0;
    d2h(c, &nf, d_nf, 8);
    CHECK(nf == NP, "n_frames %lld", (long long)nf);
    int32_t *st = malloc(4 * mp), *ist = malloc(4 * mp);
    uint32_t *olen = malloc(4 * mp);
    uint64_t *toff = malloc(8 * mp);
    uint8_t *ifo = malloc(mp * ISZ), *back = malloc(cap), *un = malloc(cap), *ref = malloc(tl);
    d2h(c, st, d_st, 4 * mp); d2h(c, ist, d_ist, 4 * mp); d2h(c, olen, d_olen, 4 * mp);
    d2h(c, toff, d_toff, 8 * mp); d2h(c, ifo, d_ifo, mp * ISZ); d2h(c, back, d_ptb, cap); d2h(c, un, d_un, cap);
    CHECK(memcmp(ifo, ifac, (uint64_t)NP * ISZ) == 0, "IFACs");
    for (int i = 0; i < NP; ++i) {
        CHECK(ist[i] == 0 && st[i] == RT_ST_OK && olen[i] == PL, "packet %d: ifac %d token %d len %u", i, ist[i],
              st[i], olen[i]);
        CHECK(memcmp(back + toff[i], pt + (uint64_t)i * PL, PL) == 0, "plaintext %d", i);
        oracle_token_encrypt(key, 64, iv + 16 * i, pt + (uint64_t)i * PL, PL, ref);
        CHECK(memcmp(un + toff[i], ref, tl) == 0, "token %d differs from the oracle's", i);
        CHECK(!slots || ((uintptr_t)d_un + toff[i] + 16) % 128 == 0, "slot %d: ciphertext not on a line", i);
    }
    for (uint64_t i = NP; i < mp; ++i) CHECK(st[i] == RT_ST_TOO_SHORT, "entry %llu past the frames: status %d",
                                           (unsigned long long)i, st[i]);
    void *bufs[] = {d_pt, d_iv, d_dh, d_ctx, d_zero, d_ifac, d_ikey, d_raw, d_mask, d_roff, d_moff, d_foff,
                    d_rlen, d_mlen, d_framed, d_fws, d_out, d_un, d_ptb, d_ifo, d_doff, d_counts, d_coff, d_toff,
                    d_dlen, d_clen, d_plen, d_tlen, d_olen, d_dst, d_ist, d_st, d_pair, d_nf, d_fields, d_dws, d_cws};
    for (unsigned k = 0; k < sizeof bufs / sizeof bufs[0]; ++k) rt_device_free(c, bufs[k]);
    free(pt); free(iv); free(dh); free(ctx); free(ifac); free(roff); free(moff); free(rlen); free(mlen); free(zero);
    free(st); free(ist); free(olen); free(toff); free(ifo); free(back); free(un); free(ref);
}

/* The measurement and copy helpers from C: rt_clock_stamps around one encrypt
 * and one decrypt launch (one launch counted each, spans and a plausible shader
 * clock), and rt_memcpy_d2h_upto with the count read on the device (clamped
 * to the destination, zero and negative counts copy nothing). */
static void clock_and_copies(rt_ctx *c, rt_keyset *k1) {
    enum { M = 1 << 16, L = 500 };
    const uint32_t tl = (uint32_t)rt_token_len(L);
    uint8_t *pt = malloc((uint64_t)M * L), *iv = malloc(16 * M);
    fill(pt, (uint64_t)M * L);
    fill(iv, 16 * M);
    uint64_t zero8[RT_CLOCK_WORDS] = {0};
    uint8_t *d_pt = h2d(c, pt, (uint64_t)M * L), *d_iv = h2d(c, iv, 16 * M);
    uint8_t *d_tok = dalloc(c, (uint64_t)M * tl), *d_back = dalloc(c, (uint64_t)M * (tl - 48));
    uint32_t *d_ol = dalloc(c, 4 * M);
    int32_t *d_st = dalloc(c, 4 * M);
    uint64_t *d_acc = h2d(c, zero8, sizeof zero8);
    CHECK(rt_clock_stamps(c, zero8) < 0, "rt_clock_stamps accepted host memory");
    RT(rt_clock_stamps(c, d_acc));
    RT(rt_encrypt_uniform(k1, d_pt, L, L, NULL, d_iv, d_tok, tl, M, NULL));
    RT(rt_decrypt_uniform(k1, d_tok, tl, tl, NULL, d_back, tl - 48, d_ol, d_st, M, NULL));
    RT(rt_clock_stamps(c, NULL));
    RT(rt_encrypt_uniform(k1, d_pt, L, L, NULL, d_iv, d_tok, tl, M, NULL));       /* not stamped */
    uint64_t w[RT_CLOCK_WORDS];
    d2h(c, w, d_acc, sizeof w);
    for (int k = RT_CLOCK_ENCRYPT; k <= RT_CLOCK_DECRYPT; ++k) {
        const uint64_t *x = w + 4 * k;
        CHECK(x[3] == 1 && x[2] >= 1 && x[0] > 0 && x[1] > 0, "clock words %d: %llu %llu %llu %llu", k,
              (unsigned long long)x[0], (unsigned long long)x[1], (unsigned long long)x[2], (unsigned long long)x[3]);
        const double ghz = (double)x[0] / (double)x[1] * 0.1;      /* ticks of 100 MHz */
        CHECK(ghz > 0.5 && ghz < 2.6, "stamped clock %.3f GHz", ghz);
    }
    /* device-sized copies into pinned memory */
    const uint64_t bytes = (uint64_t)M * (tl - 48);
    uint8_t *host = rt_host_alloc(bytes + 64), *ref = malloc(bytes);
    CHECK(host != NULL, "rt_host_alloc");
    d2h(c, ref, d_back, bytes);
    const int64_t counts[] = {0, 1, 15, 4097, (int64_t)bytes - 3, (int64_t)bytes + 100, -5};
    int64_t *d_cnt = dalloc(c, 8);
    for (unsigned t = 0; t < sizeof counts / sizeof counts[0]; ++t) {
        memset(host, 0xEE, bytes + 64);
        RT(rt_memcpy_h2d(c, d_cnt, &counts[t], 8, NULL));
        RT(rt_memcpy_d2h_upto(c, host + 3, d_back, bytes, (const uint64_t *)d_cnt, NULL));
        RT(rt_stream_sync(c, NULL));
        const uint64_t k = counts[t] <= 0 ? 0 : ((uint64_t)counts[t] < bytes ? (uint64_t)counts[t] : bytes);
        CHECK(memcmp(host + 3, ref, k) == 0, "d2h_upto %lld: bytes differ", (long long)counts[t]);
        for (uint64_t i = 0; i < 3; ++i) CHECK(host[i] == 0xEE, "d2h_upto wrote before dst");
        for (uint64_t i = 3 + k; i < bytes + 64; ++i)
            CHECK(host[i] == 0xEE, "d2h_upto %lld wrote byte %llu past the count", (long long)counts[t],
                  (unsigned long long)(i - 3));
    }
    void *bufs[] = {d_pt, d_iv, d_tok, d_back, d_ol, d_st, d_acc, d_cnt};
    for (unsigned k = 0; k < sizeof bufs / sizeof bufs[0]; ++k) rt_device_free(c, bufs[k]);
    rt_host_free(host);
    free(pt); free(iv); free(ref);
}

int main(void) {
    CHECK(rt_abi_version() == RNSTOK_ABI_VERSION, "ABI version %d", rt_abi_version());
    CHECK(rt_device_count() > 0, "no device");
    rt_ctx *c = rt_create(0);
    CHECK(c != NULL, "rt_create");
    uint8_t keys[64 * NK];
    fill(keys, sizeof keys);
    rt_keyset *ks = rt_keyset_create(c, keys, 64, NK);
    CHECK(ks != NULL, "rt_keyset_create");
    token_batch(c, ks, keys);
    rt_keyset *k1 = rt_keyset_create(c, keys, 64, 1);
    CHECK(k1 != NULL, "rt_keyset_create");
    interface_path(c, k1, keys, 0);
    interface_path(c, k1, keys, 1);
    clock_and_copies(c, k1);
    rt_keyset_destroy(k1);
    rt_keyset_destroy(ks);
    rt_destroy(c);
    printf("c_host ok: %d ragged tokens (host and device entry points), %d packets through the interface path, "
           "launch clock and device-sized copies\n", N, NP);
    return 0;
}
