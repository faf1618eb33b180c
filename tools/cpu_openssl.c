// cpu_openssl.c — the "strong CPU" row of BASELINE.md §5 item 5: the same
// token (Token.py:87-114: iv || AES-256-CBC(PKCS7(pt)) || HMAC-SHA256(sk,
// iv || ct), key = sk || ek) built on OpenSSL libcrypto (AES-NI, SHA-NI where
// the CPU has them), multithreaded over the host cores.  NOT the reference
// path (that is the pure-Python provider timed by bench.py's cpu_baseline):
// context for what a tuned CPU program does with the same work.  Per key the
// AES key schedule and the HMAC ipad/opad midstates are computed once, as
// the HIP kernels' key records do; per packet only the IV is reset.
//
// Baseline only: nothing in reticulum_amd/ loads it.  Built by
// __graft_entry__.build() into tools/libcpu_openssl.so.
#define _GNU_SOURCE
#define OPENSSL_SUPPRESS_DEPRECATED 1
#include <openssl/evp.h>
#include <openssl/sha.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef struct {
    EVP_CIPHER_CTX *enc, *dec;
    SHA256_CTX ipad, opad;
} Key;

static int key_init(Key *k, const uint8_t key[64]) {
    uint8_t pad[64];
    k->enc = EVP_CIPHER_CTX_new();
    k->dec = EVP_CIPHER_CTX_new();
    if (!k->enc || !k->dec) return -1;
    if (EVP_EncryptInit_ex(k->enc, EVP_aes_256_cbc(), NULL, key + 32, NULL) != 1) return -1;
    if (EVP_DecryptInit_ex(k->dec, EVP_aes_256_cbc(), NULL, key + 32, NULL) != 1) return -1;
    EVP_CIPHER_CTX_set_padding(k->enc, 1);   // PKCS7 (PKCS7.py:35-39)
    EVP_CIPHER_CTX_set_padding(k->dec, 0);   // unpad by hand: the reference's lenient unpad
    memset(pad, 0x36, 64);
    for (int i = 0; i < 32; ++i) pad[i] ^= key[i];
    SHA256_Init(&k->ipad);
    SHA256_Update(&k->ipad, pad, 64);
    memset(pad, 0x5c, 64);
    for (int i = 0; i < 32; ++i) pad[i] ^= key[i];
    SHA256_Init(&k->opad);
    SHA256_Update(&k->opad, pad, 64);
    return 0;
}

static void key_free(Key *k) {
    EVP_CIPHER_CTX_free(k->enc);
    EVP_CIPHER_CTX_free(k->dec);
}

static void hmac(const Key *k, const uint8_t *m, size_t n, uint8_t tag[32]) {
    SHA256_CTX c = k->ipad;
    uint8_t inner[32];
    SHA256_Update(&c, m, n);
    SHA256_Final(inner, &c);
    c = k->opad;
    SHA256_Update(&c, inner, 32);
    SHA256_Final(tag, &c);
}

// token length for L plaintext bytes: 16 + 16 * (L / 16 + 1) + 32
static int encrypt1(Key *k, const uint8_t iv[16], const uint8_t *pt, int L, uint8_t *tok) {
    int n1 = 0, n2 = 0;
    memcpy(tok, iv, 16);
    if (EVP_EncryptInit_ex(k->enc, NULL, NULL, NULL, iv) != 1) return -1;
    if (EVP_EncryptUpdate(k->enc, tok + 16, &n1, pt, L) != 1) return -1;
    if (EVP_EncryptFinal_ex(k->enc, tok + 16 + n1, &n2) != 1) return -1;
    const int ct = n1 + n2;
    hmac(k, tok, 16 + (size_t)ct, tok + 16 + ct);
    return 16 + ct + 32;
}

// returns the plaintext length, or -1 (bad tag / length / pad)
static int decrypt1(Key *k, const uint8_t *tok, int T, uint8_t *pt) {
    uint8_t tag[32];
    int n1 = 0, n2 = 0;
    if (T < 64 || ((T - 48) & 15)) return -1;
    hmac(k, tok, (size_t)T - 32, tag);
    if (memcmp(tag, tok + T - 32, 32)) return -1;
    if (EVP_DecryptInit_ex(k->dec, NULL, NULL, NULL, tok) != 1) return -1;
    if (EVP_DecryptUpdate(k->dec, pt, &n1, tok + 16, T - 48) != 1) return -1;
    if (EVP_DecryptFinal_ex(k->dec, pt + n1, &n2) != 1) return -1;
    const int n = n1 + n2, padn = pt[n - 1];
    if (padn > 16) return -1;
    return n - padn;
}

// One token (parity check against the oracle / golden vectors).
int cpu_openssl_token(const uint8_t key[64], const uint8_t iv[16], const uint8_t *pt, int L, uint8_t *tok) {
    Key k;
    if (key_init(&k, key)) return -1;
    const int r = encrypt1(&k, iv, pt, L, tok);
    key_free(&k);
    return r;
}

typedef struct {
    double seconds;
    int L, seed;
    uint64_t packets;
    double busy;
    int ok;
} Job;

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

// Round trips (encrypt, then verify + decrypt) over a ring of 1024 packets,
// one key per thread, until `seconds` have passed.
static void *worker(void *arg) {
    Job *j = (Job *)arg;
    enum { RING = 1024 };
    const int L = j->L, T = 16 + 16 * (L / 16 + 1) + 32;
    uint8_t key[64], iv[16];
    uint8_t *pt = malloc((size_t)RING * (L + 1)), *tok = malloc((size_t)T), *back = malloc((size_t)T);
    if (!pt || !tok || !back) {
        free(pt);
        free(tok);
        free(back);
        j->ok = 0;
        return NULL;
    }
    uint32_t s = 0x9E3779B9u * (uint32_t)(j->seed + 1);
#define RND() (s ^= s << 13, s ^= s >> 17, s ^= s << 5, (uint8_t)s)
    for (int i = 0; i < 64; ++i) key[i] = RND();
    for (size_t i = 0; i < (size_t)RING * (L + 1); ++i) pt[i] = RND();
    Key k;
    j->ok = key_init(&k, key) == 0;
    uint64_t n = 0;
    const double t0 = now();
    double t = t0;
    while (j->ok && t - t0 < j->seconds) {
        for (int r = 0; r < 64; ++r, ++n) {
            const uint8_t *p = pt + (size_t)(n % RING) * (L + 1);
            for (int i = 0; i < 16; ++i) iv[i] = RND();
            if (encrypt1(&k, iv, p, L, tok) != T || decrypt1(&k, tok, T, back) != L || memcmp(back, p, (size_t)L)) {
                j->ok = 0;
                break;
            }
        }
        t = now();
    }
#undef RND
    j->packets = n;
    j->busy = t - t0;
    key_free(&k);
    free(pt);
    free(tok);
    free(back);
    return NULL;
}

// Returns round trips per second over `threads` threads (sum of per-thread
// rates), or a negative value on failure; *packets_out = round trips done.
double cpu_openssl_run(int threads, double seconds, int L, uint64_t *packets_out) {
    pthread_t *th = calloc((size_t)threads, sizeof(pthread_t));
    Job *jobs = calloc((size_t)threads, sizeof(Job));
    if (!th || !jobs || threads <= 0) {
        free(th);
        free(jobs);
        return -1.0;
    }
    double rate = 0;
    uint64_t total = 0;
    int ok = 1;
    for (int i = 0; i < threads; ++i) {
        jobs[i].seconds = seconds;
        jobs[i].L = L;
        jobs[i].seed = i;
        if (pthread_create(&th[i], NULL, worker, &jobs[i])) {   // run it here instead
            worker(&jobs[i]);
            th[i] = 0;
        }
    }
    for (int i = 0; i < threads; ++i) {
        if (th[i]) pthread_join(th[i], NULL);
        ok &= jobs[i].ok;
        total += jobs[i].packets;
        if (jobs[i].busy > 0) rate += jobs[i].packets / jobs[i].busy;
    }
    free(th);
    free(jobs);
    if (packets_out) *packets_out = total;
    return ok ? rate : -1.0;
}
