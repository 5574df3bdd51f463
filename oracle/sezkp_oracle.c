/*
 * sezkp_oracle.c — CPU ORACLE (test infrastructure only; see sezkp_oracle.h).
 *
 * Plain-C restatement of the reference STARK v1 prover.  Not linked into the
 * product library; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load it (via ctypes) as the checker / CPU baseline.
 */
#include "sezkp_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef unsigned __int128 u128;

/* ========================================================================
 * Goldilocks — crates/sezkp-ffts/src/lib.rs:57-133 (u128 arithmetic, `%`)
 * ====================================================================== */
#define GL_P 0xffffffff00000001ULL

static inline uint64_t gl_add(uint64_t a, uint64_t b) { /* lib.rs:57-61 */
    u128 s = (u128)a + (u128)b;
    if (s >= (u128)GL_P) s -= GL_P;
    return (uint64_t)s;
}
static inline uint64_t gl_sub(uint64_t a, uint64_t b) { /* lib.rs:66-73 */
    if (a >= b) return a - b;
    return (uint64_t)((u128)a + (u128)GL_P - (u128)b);
}
static inline uint64_t gl_mul(uint64_t a, uint64_t b) { /* lib.rs:78-81 */
    return (uint64_t)(((u128)a * (u128)b) % (u128)GL_P);
}
static uint64_t gl_pow(uint64_t base, uint64_t e) { /* lib.rs:86-97 */
    uint64_t acc = 1;
    while (e > 0) {
        if (e & 1) acc = gl_mul(acc, base);
        base = gl_mul(base, base);
        e >>= 1;
    }
    return acc;
}
static inline uint64_t gl_inv(uint64_t a) { return gl_pow(a, GL_P - 2); } /* lib.rs:102-104 */
static inline uint64_t gl_from_u64(uint64_t x) { return x % GL_P; }         /* lib.rs:116-118 */
static inline uint64_t gl_from_i64(int64_t x) {                            /* lib.rs:109-111 rem_euclid */
    __int128 r = (__int128)x % (__int128)GL_P;
    if (r < 0) r += GL_P;
    return (uint64_t)r;
}
static uint64_t gl_root_2exp(uint32_t k) { /* lib.rs:237-242 */
    return gl_pow(7, (GL_P - 1) >> k);
}

uint64_t orc_gl_mul(uint64_t a, uint64_t b) { return gl_mul(a, b); }
uint64_t orc_gl_inv(uint64_t a) { return gl_inv(a); }
uint64_t orc_gl_root_2exp(uint32_t k) { return gl_root_2exp(k); }

/* ========================================================================
 * NTT — crates/sezkp-ffts/src/ntt.rs
 * ====================================================================== */
static size_t bitrev(size_t x, unsigned bits) { /* ntt.rs:18-25 */
    size_t y = 0;
    for (unsigned i = 0; i < bits; i++) { y = (y << 1) | (x & 1); x >>= 1; }
    return y;
}
static void bit_reverse_permute(uint64_t *a, size_t n) { /* ntt.rs:29-39 */
    unsigned bits = 0;
    while (((size_t)1 << bits) < n) bits++;
    for (size_t i = 0; i < n; i++) {
        size_t j = bitrev(i, bits);
        if (j > i) { uint64_t t = a[i]; a[i] = a[j]; a[j] = t; }
    }
}
/* ntt.rs:79-111 (forward) and 117-155 (inverse): DIT with per-stage twiddles */
static void ntt_core(uint64_t *a, size_t n, int inverse) {
    if (n <= 1) return;
    bit_reverse_permute(a, n);
    uint64_t *ws = (uint64_t *)malloc(sizeof(uint64_t) * (n / 2));
    unsigned stage = 1;
    for (size_t len = 2; len <= n; len <<= 1, stage++) {
        size_t half = len / 2;
        uint64_t w_len = gl_root_2exp(stage);       /* ntt.rs:42-56 */
        if (inverse) w_len = gl_inv(w_len);          /* ntt.rs:59-74 */
        uint64_t w = 1;
        for (size_t i = 0; i < half; i++) { ws[i] = w; w = gl_mul(w, w_len); }
        /* butterflies of one stage are independent (OpenMP build: cpu_baseline) */
        #pragma omp parallel for schedule(static) if (n >= 4096)
        for (size_t t = 0; t < n / 2; t++) {
            size_t j = (t / half) * len, i = t % half;
            uint64_t u = a[j + i];
            uint64_t v = gl_mul(a[j + i + half], ws[i]);
            a[j + i] = gl_add(u, v);
            a[j + i + half] = gl_sub(u, v);
        }
    }
    free(ws);
    if (inverse) { /* ntt.rs:151-154 */
        uint64_t inv_n = gl_inv(gl_from_u64((uint64_t)n));
        #pragma omp parallel for schedule(static) if (n >= 4096)
        for (size_t i = 0; i < n; i++) a[i] = gl_mul(a[i], inv_n);
    }
}
void orc_ntt_forward(uint64_t *a, size_t n) { ntt_core(a, n, 0); }
void orc_ntt_inverse(uint64_t *a, size_t n) { ntt_core(a, n, 1); }

/* coset.rs:85-102: scale by shift^j, zero-pad/truncate to 2^k, forward NTT */
void orc_coset_lde(const uint64_t *coeffs, size_t m, uint32_t k_log2, uint64_t shift, uint64_t *out) {
    size_t n = (size_t)1 << k_log2;
    memset(out, 0, n * sizeof(uint64_t));
    if (m > n) m = n;
    #pragma omp parallel for schedule(static) if (m >= 4096)
    for (size_t c0 = 0; c0 < m; c0 += 1024) {  /* chunks restart shift^j from shift^c0 */
        uint64_t pw = gl_pow(shift, c0);
        for (size_t j = c0; j < m && j < c0 + 1024; j++) { out[j] = gl_mul(coeffs[j], pw); pw = gl_mul(pw, shift); }
    }
    ntt_core(out, n, 0);
}

/* benches/ntt.rs:21-34 */
void orc_det_vec(uint64_t *out, size_t n, uint64_t seed) {
    const uint64_t A = 1664525ULL, C = 1013904223ULL, M = 1ULL << 32;
    uint64_t a = A * seed + C;
    for (size_t i = 0; i < n; i++) {
        a = (a * A + C) % M;
        out[i] = gl_from_u64(a ^ ((uint64_t)i * 0x9E3779B97F4A7C15ULL));
    }
}

/* ========================================================================
 * BLAKE3 — restated from the published specification (hash mode, XOF)
 * ====================================================================== */
#define B3_CHUNK_START 1u
#define B3_CHUNK_END 2u
#define B3_PARENT 4u
#define B3_ROOT 8u
static const uint32_t B3_IV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                                  0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
static const uint8_t B3_PERM[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};

static inline uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
static inline void b3_g(uint32_t *s, int a, int b, int c, int d, uint32_t mx, uint32_t my) {
    s[a] = s[a] + s[b] + mx; s[d] = rotr32(s[d] ^ s[a], 16);
    s[c] = s[c] + s[d];      s[b] = rotr32(s[b] ^ s[c], 12);
    s[a] = s[a] + s[b] + my; s[d] = rotr32(s[d] ^ s[a], 8);
    s[c] = s[c] + s[d];      s[b] = rotr32(s[b] ^ s[c], 7);
}
static void b3_compress(const uint32_t cv[8], const uint32_t block[16], uint64_t counter,
                        uint32_t block_len, uint32_t flags, uint32_t out[16]) {
    uint32_t s[16] = {cv[0], cv[1], cv[2], cv[3], cv[4], cv[5], cv[6], cv[7],
                      B3_IV[0], B3_IV[1], B3_IV[2], B3_IV[3],
                      (uint32_t)counter, (uint32_t)(counter >> 32), block_len, flags};
    uint32_t m[16], t[16];
    memcpy(m, block, 64);
    for (int r = 0; r < 7; r++) {
        b3_g(s, 0, 4, 8, 12, m[0], m[1]);
        b3_g(s, 1, 5, 9, 13, m[2], m[3]);
        b3_g(s, 2, 6, 10, 14, m[4], m[5]);
        b3_g(s, 3, 7, 11, 15, m[6], m[7]);
        b3_g(s, 0, 5, 10, 15, m[8], m[9]);
        b3_g(s, 1, 6, 11, 12, m[10], m[11]);
        b3_g(s, 2, 7, 8, 13, m[12], m[13]);
        b3_g(s, 3, 4, 9, 14, m[14], m[15]);
        if (r < 6) {
            for (int i = 0; i < 16; i++) t[i] = m[B3_PERM[i]];
            memcpy(m, t, 64);
        }
    }
    for (int i = 0; i < 8; i++) { out[i] = s[i] ^ s[i + 8]; out[i + 8] = s[i + 8] ^ cv[i]; }
}
static void b3_words_from_bytes(const uint8_t *b, uint32_t w[16]) {
    for (int i = 0; i < 16; i++)
        w[i] = (uint32_t)b[4 * i] | ((uint32_t)b[4 * i + 1] << 8) | ((uint32_t)b[4 * i + 2] << 16) |
               ((uint32_t)b[4 * i + 3] << 24);
}

typedef struct {
    uint32_t cv[8];
    uint64_t chunk_counter;
    uint8_t block[64];
    uint32_t block_len;
    uint32_t blocks_compressed;
} b3_chunk;
typedef struct {
    b3_chunk chunk;
    uint32_t cv_stack[64][8];
    uint32_t cv_len;
} b3_hasher;

static void b3_chunk_init(b3_chunk *c, uint64_t counter) {
    memcpy(c->cv, B3_IV, 32);
    c->chunk_counter = counter;
    memset(c->block, 0, 64);
    c->block_len = 0;
    c->blocks_compressed = 0;
}
static uint32_t b3_chunk_len(const b3_chunk *c) { return 64 * c->blocks_compressed + c->block_len; }
static void b3_chunk_update(b3_chunk *c, const uint8_t *in, size_t len) {
    while (len > 0) {
        if (c->block_len == 64) {
            uint32_t w[16], o[16];
            b3_words_from_bytes(c->block, w);
            b3_compress(c->cv, w, c->chunk_counter, 64,
                        c->blocks_compressed == 0 ? B3_CHUNK_START : 0, o);
            memcpy(c->cv, o, 32);
            c->blocks_compressed++;
            memset(c->block, 0, 64);
            c->block_len = 0;
        }
        size_t take = 64 - c->block_len;
        if (take > len) take = len;
        memcpy(c->block + c->block_len, in, take);
        c->block_len += (uint32_t)take;
        in += take;
        len -= take;
    }
}
typedef struct {
    uint32_t cv[8];
    uint32_t block[16];
    uint64_t counter;
    uint32_t block_len;
    uint32_t flags;
} b3_output;
static b3_output b3_chunk_output(const b3_chunk *c) {
    b3_output o;
    memcpy(o.cv, c->cv, 32);
    b3_words_from_bytes(c->block, o.block);
    o.counter = c->chunk_counter;
    o.block_len = c->block_len;
    o.flags = (c->blocks_compressed == 0 ? B3_CHUNK_START : 0) | B3_CHUNK_END;
    return o;
}
static void b3_output_cv(const b3_output *o, uint32_t cv[8]) {
    uint32_t t[16];
    b3_compress(o->cv, o->block, o->counter, o->block_len, o->flags, t);
    memcpy(cv, t, 32);
}
static b3_output b3_parent_output(const uint32_t l[8], const uint32_t r[8]) {
    b3_output o;
    memcpy(o.cv, B3_IV, 32);
    memcpy(o.block, l, 32);
    memcpy(o.block + 8, r, 32);
    o.counter = 0;
    o.block_len = 64;
    o.flags = B3_PARENT;
    return o;
}
static void b3_init(b3_hasher *h) { b3_chunk_init(&h->chunk, 0); h->cv_len = 0; }
static void b3_update(b3_hasher *h, const uint8_t *in, size_t len) {
    while (len > 0) {
        if (b3_chunk_len(&h->chunk) == 1024) {
            b3_output o = b3_chunk_output(&h->chunk);
            uint32_t cv[8];
            b3_output_cv(&o, cv);
            uint64_t total = h->chunk.chunk_counter + 1;
            while ((total & 1) == 0) {
                h->cv_len--;
                b3_output p = b3_parent_output(h->cv_stack[h->cv_len], cv);
                b3_output_cv(&p, cv);
                total >>= 1;
            }
            memcpy(h->cv_stack[h->cv_len++], cv, 32);
            b3_chunk_init(&h->chunk, h->chunk.chunk_counter + 1);
        }
        size_t want = 1024 - b3_chunk_len(&h->chunk);
        size_t take = want < len ? want : len;
        b3_chunk_update(&h->chunk, in, take);
        in += take;
        len -= take;
    }
}
static void b3_finalize(const b3_hasher *h, uint8_t *out, size_t out_len) {
    b3_output o = b3_chunk_output(&h->chunk);
    uint32_t rem = h->cv_len;
    while (rem > 0) {
        rem--;
        uint32_t cv[8];
        b3_output_cv(&o, cv);
        o = b3_parent_output(h->cv_stack[rem], cv);
    }
    uint64_t ctr = 0;
    while (out_len > 0) {
        uint32_t w[16];
        b3_compress(o.cv, o.block, ctr, o.block_len, o.flags | B3_ROOT, w);
        for (int i = 0; i < 16 && out_len > 0; i++)
            for (int k = 0; k < 4 && out_len > 0; k++) { *out++ = (uint8_t)(w[i] >> (8 * k)); out_len--; }
        ctr++;
    }
}
void orc_blake3(const uint8_t *in, size_t len, uint8_t *out, size_t out_len) {
    b3_hasher h;
    b3_init(&h);
    b3_update(&h, in, len);
    b3_finalize(&h, out, out_len);
}

/* ========================================================================
 * Transcript — crates/sezkp-crypto/src/lib.rs:74-123
 * ====================================================================== */
struct orc_transcript { b3_hasher st; };
static void u32le(uint8_t *p, uint32_t x) { for (int i = 0; i < 4; i++) p[i] = (uint8_t)(x >> (8 * i)); }
static void u64le(uint8_t *p, uint64_t x) { for (int i = 0; i < 8; i++) p[i] = (uint8_t)(x >> (8 * i)); }
static uint64_t rd64le(const uint8_t *p) { uint64_t x = 0; for (int i = 7; i >= 0; i--) x = (x << 8) | p[i]; return x; }

static void tr_init(orc_transcript *t, const char *domain) { /* lib.rs:81-88 */
    uint8_t l[4];
    b3_init(&t->st);
    b3_update(&t->st, (const uint8_t *)"sezkp.transcript.v0", 19);
    u32le(l, (uint32_t)strlen(domain));
    b3_update(&t->st, l, 4);
    b3_update(&t->st, (const uint8_t *)domain, strlen(domain));
}
static void tr_absorb(orc_transcript *t, const char *label, const uint8_t *bytes, size_t len) { /* 92-100 */
    uint8_t l[4];
    b3_update(&t->st, (const uint8_t *)"absorb", 6);
    u32le(l, (uint32_t)strlen(label));
    b3_update(&t->st, l, 4);
    b3_update(&t->st, (const uint8_t *)label, strlen(label));
    u32le(l, (uint32_t)len);
    b3_update(&t->st, l, 4);
    b3_update(&t->st, bytes, len);
}
static void tr_absorb_u64(orc_transcript *t, const char *label, uint64_t x) { /* 53-55 */
    uint8_t b[8];
    u64le(b, x);
    tr_absorb(t, label, b, 8);
}
static void tr_challenge(orc_transcript *t, const char *label, uint8_t *out, size_t n) { /* 102-123 */
    uint8_t l[4];
    b3_hasher st = t->st;
    b3_update(&st, (const uint8_t *)"challenge", 9);
    u32le(l, (uint32_t)strlen(label));
    b3_update(&st, l, 4);
    b3_update(&st, (const uint8_t *)label, strlen(label));
    b3_finalize(&st, out, n);
    b3_update(&t->st, (const uint8_t *)"after_challenge", 15);
    b3_update(&t->st, l, 4);
    b3_update(&t->st, (const uint8_t *)label, strlen(label));
}
orc_transcript *orc_tr_new(const char *domain) {
    orc_transcript *t = (orc_transcript *)malloc(sizeof(orc_transcript));
    tr_init(t, domain);
    return t;
}
void orc_tr_free(orc_transcript *t) { free(t); }
void orc_tr_absorb(orc_transcript *t, const char *label, const uint8_t *bytes, size_t len) { tr_absorb(t, label, bytes, len); }
void orc_tr_absorb_u64(orc_transcript *t, const char *label, uint64_t x) { tr_absorb_u64(t, label, x); }
void orc_tr_challenge(orc_transcript *t, const char *label, uint8_t *out, size_t n) { tr_challenge(t, label, out, n); }

/* ========================================================================
 * Merkle helpers — crates/sezkp-stark/src/v1/merkle.rs
 * ====================================================================== */
static void hash2(const uint8_t *l, const uint8_t *r, uint8_t *out) { /* merkle.rs:58-61, fri_stream.rs:45-50 */
    uint8_t buf[64];
    memcpy(buf, l, 32);
    memcpy(buf + 32, r, 32);
    orc_blake3(buf, 64, out, 32);
}
void orc_hash_leaf_u64(uint64_t v, uint8_t out[32]) { /* merkle.rs:150-160 */
    uint8_t b[8];
    u64le(b, v);
    orc_blake3(b, 8, out, 32);
}
void orc_hash_leaf_labeled(uint64_t v, const char *label, uint8_t out[32]) { /* merkle.rs:132-147 */
    uint8_t buf[128];
    size_t ll = strlen(label), p = 0;
    memcpy(buf, "col_leaf", 8); p = 8;
    u32le(buf + p, (uint32_t)ll); p += 4;
    memcpy(buf + p, label, ll); p += ll;
    u64le(buf + p, v); p += 8;
    orc_blake3(buf, p, out, 32);
}

/* MerkleTree::from_leaves (merkle.rs:46-71): all levels, odd promotion.
 * Levels stored bottom-up; returns node array, level offsets in lvl_off. */
typedef struct {
    uint8_t *nodes;     /* concatenated levels, 32 B each */
    size_t *lvl_off;    /* start index (in nodes) of each level */
    size_t *lvl_len;
    size_t n_levels;
} mtree;
static void mtree_build(mtree *t, const uint8_t *leaves, size_t n) {
    static const uint8_t zero[32] = {0};
    if (n == 0) { leaves = zero; n = 1; } /* merkle.rs:48-50 */
    size_t total = 0, len = n, levels = 0;
    while (1) { total += len; levels++; if (len == 1) break; len = (len + 1) / 2; }
    t->nodes = (uint8_t *)malloc(total * 32);
    t->lvl_off = (size_t *)malloc(levels * sizeof(size_t));
    t->lvl_len = (size_t *)malloc(levels * sizeof(size_t));
    t->n_levels = levels;
    memcpy(t->nodes, leaves, n * 32);
    t->lvl_off[0] = 0;
    t->lvl_len[0] = n;
    for (size_t l = 1; l < levels; l++) {
        size_t po = t->lvl_off[l - 1], pl = t->lvl_len[l - 1];
        size_t o = po + pl, nl = (pl + 1) / 2;
        t->lvl_off[l] = o;
        t->lvl_len[l] = nl;
        #pragma omp parallel for schedule(static) if (pl >= 2048)
        for (size_t i = 0; i < pl; i += 2) {
            if (i + 1 < pl) hash2(t->nodes + 32 * (po + i), t->nodes + 32 * (po + i + 1), t->nodes + 32 * (o + i / 2));
            else memcpy(t->nodes + 32 * (o + i / 2), t->nodes + 32 * (po + i), 32);
        }
    }
}
static const uint8_t *mtree_root(const mtree *t) { return t->nodes + 32 * t->lvl_off[t->n_levels - 1]; }
/* MerkleTree::open (merkle.rs:80-108): siblings bottom->top; returns count */
static size_t mtree_open(const mtree *t, size_t idx, uint8_t *sibs) {
    size_t cnt = 0;
    idx %= t->lvl_len[0];
    for (size_t l = 0; l + 1 < t->n_levels; l++) {
        size_t len = t->lvl_len[l];
        size_t sib = ((idx ^ 1) < len) ? (idx ^ 1) : idx;
        memcpy(sibs + 32 * cnt, t->nodes + 32 * (t->lvl_off[l] + sib), 32);
        cnt++;
        idx >>= 1;
    }
    return cnt;
}
static void mtree_free(mtree *t) { free(t->nodes); free(t->lvl_off); free(t->lvl_len); }

void orc_merkle_root(const uint8_t *leaves32, size_t n, uint8_t root[32]) {
    mtree t;
    mtree_build(&t, leaves32, n);
    memcpy(root, mtree_root(&t), 32);
    mtree_free(&t);
}

/* MerkleTree::from_leaves (merkle.rs:46-71): every level bottom->top into
 * out (level 0 = the leaves; n = 0 is one zero leaf); returns the node count */
size_t orc_merkle_nodes(const uint8_t *leaves32, size_t n, uint8_t *out) {
    mtree t;
    mtree_build(&t, leaves32, n);
    size_t total = t.lvl_off[t.n_levels - 1] + 1;
    if (out) memcpy(out, t.nodes, 32 * total);
    mtree_free(&t);
    return total;
}

/* MerkleTree::open (merkle.rs:80-108) for q indices: q * depth siblings */
size_t orc_merkle_open(const uint8_t *leaves32, size_t n, const uint64_t *idx, size_t q, uint8_t *sibs) {
    mtree t;
    mtree_build(&t, leaves32, n);
    size_t depth = t.n_levels - 1;
    for (size_t i = 0; i < q; i++) mtree_open(&t, (size_t)idx[i], sibs + 32 * depth * i);
    mtree_free(&t);
    return depth;
}

/* StreamingLayerBuilder (fri_stream.rs:55-121) */
typedef struct {
    uint8_t (*stack)[32];
    uint8_t *has;
    size_t cap, len, seen;
} slb;
static void slb_init(slb *s) { s->cap = 72; s->stack = malloc(32 * s->cap); s->has = calloc(s->cap, 1); s->len = 0; s->seen = 0; }
static void slb_absorb_leaf(slb *s, const uint8_t leaf[32]) { /* fri_stream.rs:75-95 */
    uint8_t cur[32];
    memcpy(cur, leaf, 32);
    s->seen++;
    size_t lvl = 0;
    for (;;) {
        if (s->len <= lvl) { s->has[s->len] = 0; s->len++; }
        if (s->has[lvl]) {
            uint8_t t[32];
            hash2(s->stack[lvl], cur, t);
            s->has[lvl] = 0;
            memcpy(cur, t, 32);
            lvl++;
        } else {
            memcpy(s->stack[lvl], cur, 32);
            s->has[lvl] = 1;
            break;
        }
    }
}
static void slb_finalize(slb *s, uint8_t out[32]) { /* fri_stream.rs:99-121 */
    int have = 0;
    uint8_t cur[32];
    for (size_t l = s->len; l-- > 0;) {
        if (!s->has[l]) continue;
        if (!have) { memcpy(cur, s->stack[l], 32); have = 1; }
        else { uint8_t t[32]; hash2(s->stack[l], cur, t); memcpy(cur, t, 32); }
    }
    if (!have) memset(cur, 0, 32);
    memcpy(out, cur, 32);
    free(s->stack);
    free(s->has);
}

/* ========================================================================
 * Manifest — crates/sezkp-merkle/src/lib.rs:85-208
 * ====================================================================== */
void orc_manifest_leaf_hash(const orc_blocks *b, uint32_t k, uint8_t out[32]) { /* lib.rs:85-117 */
    size_t tau = b->tau;
    size_t cap = 2 + 4 + 8 + 8 + 2 + 2 + 8 + 8 + 8 + 16 * tau + 8 * tau + 8;
    uint8_t *buf = (uint8_t *)malloc(cap), *p = buf;
    p[0] = (uint8_t)b->version[k]; p[1] = (uint8_t)(b->version[k] >> 8); p += 2;
    u32le(p, b->block_id[k]); p += 4;
    u64le(p, b->step_lo[k]); p += 8;
    u64le(p, b->step_hi[k]); p += 8;
    p[0] = (uint8_t)b->ctrl_in[k]; p[1] = (uint8_t)(b->ctrl_in[k] >> 8); p += 2;
    p[0] = (uint8_t)b->ctrl_out[k]; p[1] = (uint8_t)(b->ctrl_out[k] >> 8); p += 2;
    u64le(p, (uint64_t)b->in_head_in[k]); p += 8;
    u64le(p, (uint64_t)b->in_head_out[k]); p += 8;
    u64le(p, (uint64_t)tau); p += 8;
    for (size_t r = 0; r < tau; r++) {
        u64le(p, (uint64_t)b->win_left[k * tau + r]); p += 8;
        u64le(p, (uint64_t)b->win_right[k * tau + r]); p += 8;
    }
    for (size_t r = 0; r < tau; r++) { u32le(p, b->off_in[k * tau + r]); p += 4; }
    for (size_t r = 0; r < tau; r++) { u32le(p, b->off_out[k * tau + r]); p += 4; }
    u64le(p, b->step_start[k + 1] - b->step_start[k]); p += 8;
    orc_blake3(buf, (size_t)(p - buf), out, 32);
    free(buf);
}
void orc_manifest_root(const orc_blocks *b, uint8_t out[32]) { /* lib.rs:140-157, 214-222 */
    if (b->n_blocks == 0) { memset(out, 0, 32); return; }
    size_t n = b->n_blocks;
    uint8_t *lv = (uint8_t *)malloc(32 * n);
    for (uint32_t k = 0; k < b->n_blocks; k++) orc_manifest_leaf_hash(b, k, lv + 32 * k);
    while (n > 1) {
        size_t m = 0;
        for (size_t i = 0; i < n; i += 2) {
            if (i + 1 < n) hash2(lv + 32 * i, lv + 32 * (i + 1), lv + 32 * m);
            else memmove(lv + 32 * m, lv + 32 * i, 32);
            m++;
        }
        n = m;
    }
    memcpy(out, lv, 32);
    free(lv);
}
void orc_manifest_frontier_root(const uint8_t *leaves32, size_t n, uint8_t out[32]) { /* lib.rs:167-208 */
    uint8_t slots[72][32];
    uint8_t has[72] = {0};
    size_t nslots = 0;
    for (size_t i = 0; i < n; i++) {
        uint8_t h[32];
        memcpy(h, leaves32 + 32 * i, 32);
        size_t lvl = 0;
        for (;;) {
            if (nslots <= lvl) { has[nslots] = 0; nslots = lvl + 1; }
            if (!has[lvl]) { memcpy(slots[lvl], h, 32); has[lvl] = 1; break; }
            uint8_t t[32];
            has[lvl] = 0;
            hash2(slots[lvl], h, t);
            memcpy(h, t, 32);
            lvl++;
        }
    }
    int have = 0;
    uint8_t acc[32];
    for (size_t l = nslots; l-- > 0;) {
        if (!has[l]) continue;
        if (!have) { memcpy(acc, slots[l], 32); have = 1; }
        else { uint8_t t[32]; hash2(acc, slots[l], t); memcpy(acc, t, 32); } /* merkle_parent(higher, node) */
    }
    if (!have) memset(acc, 0, 32);
    memcpy(out, acc, 32);
}

/* ========================================================================
 * v0 StarkIOP — sezkp-stark/src/lib.rs:66-95, commit.rs:47-90, witness.rs:33-105
 * ====================================================================== */
int orc_v0_proof(const orc_blocks *b, const uint8_t manifest_root[32], uint8_t out64[64], uint64_t *n_rows_out) {
    uint8_t root[32];
    uint64_t n_rows = 0;
    size_t tau = b->tau;
    if (b->n_blocks == 0) {
        orc_transcript t;
        tr_init(&t, "sezkp-stark/v0/row-stream/empty");
        tr_challenge(&t, "root", root, 32);
        tau = 0;
    } else {
        orc_transcript t;
        tr_init(&t, "sezkp-stark/v0/row-stream");
        tr_absorb_u64(&t, "tau", tau);
        size_t row_len = 1 + 2 * tau, chunk_rows = 4096;
        uint8_t *buf = (uint8_t *)malloc(row_len * chunk_rows);
        size_t rows = 0, total = b->step_start[b->n_blocks];
        for (size_t s = 0; s < total; s++) {
            uint8_t *p = buf + rows * row_len;
            p[0] = (uint8_t)b->input_mv[s];
            for (size_t r = 0; r < tau; r++) {
                p[1 + 2 * r] = (uint8_t)(b->mv[s * tau + r] + 1);
                p[2 + 2 * r] = b->has_write[s * tau + r] ? 1 : 0;
            }
            rows++;
            if (rows == chunk_rows) { tr_absorb(&t, "rows", buf, rows * row_len); n_rows += rows; rows = 0; }
        }
        if (rows) { tr_absorb(&t, "rows", buf, rows * row_len); n_rows += rows; }
        free(buf);
        tr_challenge(&t, "root", root, 32);
    }
    orc_transcript t;
    tr_init(&t, "sezkp-stark-v0");
    tr_absorb(&t, "manifest_root", manifest_root, 32);
    tr_absorb(&t, "commit_root", root, 32);
    tr_absorb_u64(&t, "n_rows", n_rows);
    tr_absorb_u64(&t, "tau", tau);
    tr_challenge(&t, "alpha", out64, 32);
    tr_challenge(&t, "beta", out64 + 32, 32);
    if (n_rows_out) *n_rows_out = n_rows;
    return 0;
}

/* ========================================================================
 * v1 trace columns — columns.rs:252-365, openings.rs:89-273
 * ====================================================================== */
enum { K_MV = 0, K_WFLAG, K_WSYM, K_HEAD, K_WINLEN, K_INOFF, K_OUTOFF };
static const char *KIND_NAME[7] = {"mv", "wflag", "wsym", "head", "winlen", "in_off", "out_off"};

/* all_labels (openings.rs:89-116) */
static void label_of(size_t c, size_t tau, char *out) {
    if (c == 0) { strcpy(out, "input_mv"); return; }
    if (c == 1) { strcpy(out, "is_first"); return; }
    if (c == 2) { strcpy(out, "is_last"); return; }
    size_t k = (c - 3) / tau, r = (c - 3) % tau;
    sprintf(out, "%s_%zu", KIND_NAME[k], r);
}

typedef struct {
    size_t n, tau, ncols;
    /* column-major values: col[c*n + i], canonical field elements */
    uint64_t *col;
    /* TraceColumns aux: head as i64 not needed (field values suffice) */
} trace_cols;

/* Build all 3+7tau committed columns (RowIter semantics, openings.rs:227-273,
 * identical to TraceColumns::build columns.rs:252-365). */
static int build_cols(const orc_blocks *b, trace_cols *tc, char *err, size_t err_len) {
    size_t tau = b->tau, n = 0;
    for (uint32_t k = 0; k < b->n_blocks; k++) {
        uint64_t len = b->step_hi[k] - b->step_lo[k] + 1;
        if (len != b->step_start[k + 1] - b->step_start[k]) {
            snprintf(err, err_len, "block %u: step_hi-step_lo+1=%llu but %llu steps", k,
                     (unsigned long long)len, (unsigned long long)(b->step_start[k + 1] - b->step_start[k]));
            return -2;
        }
        n += len;
    }
    tc->n = n;
    tc->tau = tau;
    tc->ncols = 3 + 7 * tau;
    tc->col = (uint64_t *)calloc(tc->ncols * (n ? n : 1), sizeof(uint64_t));
    int64_t *heads = (int64_t *)calloc(tau ? tau : 1, sizeof(int64_t));
    size_t row = 0;
    for (uint32_t k = 0; k < b->n_blocks; k++) {
        size_t len = (size_t)(b->step_start[k + 1] - b->step_start[k]);
        for (size_t r = 0; r < tau; r++) heads[r] = 0;
        for (size_t j = 0; j < len; j++, row++) {
            size_t s = (size_t)b->step_start[k] + j;
            tc->col[0 * n + row] = gl_from_i64(b->input_mv[s]);
            tc->col[1 * n + row] = (j == 0) ? 1 : 0;
            tc->col[2 * n + row] = (j + 1 == len) ? 1 : 0;
            for (size_t r = 0; r < tau; r++) {
                size_t o = s * tau + r;
                int64_t left = b->win_left[k * tau + r], right = b->win_right[k * tau + r];
                int64_t d = right - left;
                uint64_t wl = (uint64_t)(d < 0 ? -d : d) + 1;
                heads[r] += b->mv[o];
                tc->col[(3 + K_MV * tau + r) * n + row] = gl_from_i64(b->mv[o]);
                tc->col[(3 + K_WFLAG * tau + r) * n + row] = b->has_write[o] ? 1 : 0;
                tc->col[(3 + K_WSYM * tau + r) * n + row] = b->has_write[o] ? gl_from_u64(b->wsym[o]) : 0;
                tc->col[(3 + K_HEAD * tau + r) * n + row] = gl_from_i64(heads[r]);
                tc->col[(3 + K_WINLEN * tau + r) * n + row] = gl_from_u64(wl);
                tc->col[(3 + K_INOFF * tau + r) * n + row] = gl_from_u64(b->off_in[k * tau + r]);
                tc->col[(3 + K_OUTOFF * tau + r) * n + row] = gl_from_u64(b->off_out[k * tau + r]);
            }
        }
    }
    free(heads);
    return 0;
}
#define COL(tc, c, i) ((tc)->col[(c) * (tc)->n + (i)])

/* ========================================================================
 * AIR composition — air.rs:49-136 (compose_row + compose_boundary)
 * ====================================================================== */
typedef struct {
    uint64_t bool_flag, mv_domain, head_update, head_bits_bool, head_reconstruct,
        slack_bits_bool, slack_reconstruct, sym_bits_bool, sym_reconstruct, boundary_first, boundary_last;
} alphas_t;

static uint64_t compose_row(const trace_cols *tc, size_t i, const alphas_t *a) {
    uint64_t acc = 0;
    size_t tau = tc->tau, n = tc->n;
    for (size_t r = 0; r < tau; r++) {
        uint64_t mv = COL(tc, 3 + K_MV * tau + r, i);
        uint64_t flg = COL(tc, 3 + K_WFLAG * tau + r, i);
        uint64_t head = COL(tc, 3 + K_HEAD * tau + r, i);
        size_t ip1 = (i + 1) % n;
        uint64_t head_next = COL(tc, 3 + K_HEAD * tau + r, ip1);
        uint64_t mv_next = COL(tc, 3 + K_MV * tau + r, ip1);
        /* C1 */
        acc = gl_add(acc, gl_mul(gl_mul(a->bool_flag, flg), gl_sub(flg, 1)));
        /* C2 */
        acc = gl_add(acc, gl_mul(gl_mul(gl_mul(a->mv_domain, mv), gl_sub(mv, 1)), gl_add(mv, 1)));
        /* C3 */
        uint64_t oml = gl_sub(1, COL(tc, 2, i));
        acc = gl_add(acc, gl_mul(gl_mul(a->head_update, oml), gl_sub(gl_sub(head_next, head), mv_next)));
        /* head bits (columns.rs:329-334) */
        uint64_t hsum = 0, hb = 0, pw = 1;
        for (int k = 0; k < 16; k++) {
            uint64_t bit = (head >> k) & 1;
            hb = gl_add(hb, gl_mul(bit, gl_sub(bit, 1)));
            hsum = gl_add(hsum, gl_mul(bit, pw));
            pw = gl_mul(pw, 2);
        }
        acc = gl_add(acc, gl_mul(gl_mul(a->head_bits_bool, flg), hb));
        acc = gl_add(acc, gl_mul(gl_mul(a->head_reconstruct, flg), gl_sub(head, hsum)));
        /* slack bits (columns.rs:335-341) */
        uint64_t winlen = COL(tc, 3 + K_WINLEN * tau + r, i);
        uint64_t slack = gl_sub(gl_sub(winlen, 1), head);
        uint64_t ssum = 0, sb = 0;
        pw = 1;
        for (int k = 0; k < 16; k++) {
            uint64_t bit = (slack >> k) & 1;
            sb = gl_add(sb, gl_mul(bit, gl_sub(bit, 1)));
            ssum = gl_add(ssum, gl_mul(bit, pw));
            pw = gl_mul(pw, 2);
        }
        acc = gl_add(acc, gl_mul(gl_mul(a->slack_bits_bool, flg), sb));
        acc = gl_add(acc, gl_mul(gl_mul(a->slack_reconstruct, flg), gl_sub(slack, ssum)));
        /* symbol bits (columns.rs:323-328) */
        uint64_t wsym = COL(tc, 3 + K_WSYM * tau + r, i);
        uint64_t ysum = 0, yb = 0;
        pw = 1;
        for (int k = 0; k < 4; k++) {
            uint64_t bit = (wsym >> k) & 1;
            yb = gl_add(yb, gl_mul(bit, gl_sub(bit, 1)));
            ysum = gl_add(ysum, gl_mul(bit, pw));
            pw = gl_mul(pw, 2);
        }
        acc = gl_add(acc, gl_mul(gl_mul(a->sym_bits_bool, flg), yb));
        acc = gl_add(acc, gl_mul(gl_mul(a->sym_reconstruct, flg), gl_sub(wsym, ysum)));
    }
    return acc;
}
static uint64_t compose_boundary(const trace_cols *tc, size_t i, const alphas_t *a) {
    uint64_t acc = 0;
    size_t tau = tc->tau;
    uint64_t is_first = COL(tc, 1, i), is_last = COL(tc, 2, i);
    for (size_t r = 0; r < tau; r++) {
        uint64_t head = COL(tc, 3 + K_HEAD * tau + r, i);
        uint64_t mv = COL(tc, 3 + K_MV * tau + r, i);
        uint64_t off_in = COL(tc, 3 + K_INOFF * tau + r, i);
        uint64_t off_out = COL(tc, 3 + K_OUTOFF * tau + r, i);
        acc = gl_add(acc, gl_mul(gl_mul(a->boundary_first, is_first), gl_sub(gl_sub(head, mv), off_in)));
        acc = gl_add(acc, gl_mul(gl_mul(a->boundary_last, is_last), gl_sub(head, off_out)));
    }
    return acc;
}

/* ========================================================================
 * Column commitments — openings.rs:306-398 (chunked, 1024 rows per chunk)
 * ====================================================================== */
#define COL_CHUNK 1024
typedef struct {
    size_t n_chunks;
    uint8_t *chunk_roots; /* [n_chunks*32] */
    uint8_t root[32];
} col_commit;

static void chunk_leaves(const trace_cols *tc, size_t c, const char *label, size_t start, size_t end, uint8_t *lv) {
    for (size_t i = start; i < end; i++) orc_hash_leaf_labeled(COL(tc, c, i), label, lv + 32 * (i - start));
}
static void commit_column(const trace_cols *tc, size_t c, col_commit *cc) {
    char label[64];
    label_of(c, tc->tau, label);
    size_t n = tc->n;
    cc->n_chunks = (n + COL_CHUNK - 1) / COL_CHUNK;
    cc->chunk_roots = (uint8_t *)malloc(32 * (cc->n_chunks ? cc->n_chunks : 1));
    uint8_t *lv = (uint8_t *)malloc(32 * COL_CHUNK);
    for (size_t ch = 0; ch < cc->n_chunks; ch++) {
        size_t s = ch * COL_CHUNK, e = s + COL_CHUNK < n ? s + COL_CHUNK : n;
        chunk_leaves(tc, c, label, s, e, lv);
        orc_merkle_root(lv, e - s, cc->chunk_roots + 32 * ch);
    }
    free(lv);
    orc_merkle_root(cc->chunk_roots, cc->n_chunks, cc->root); /* empty -> zero leaf */
}

/* ========================================================================
 * Byte buffer + bincode 1.3.3 (fixint LE) writer — proof.rs:80-98
 * ====================================================================== */
typedef struct { uint8_t *p; size_t len, cap; } bbuf;
static void bb_put(bbuf *b, const void *d, size_t n) {
    if (b->len + n > b->cap) {
        size_t nc = b->cap ? b->cap * 2 : 4096;
        while (nc < b->len + n) nc *= 2;
        b->p = (uint8_t *)realloc(b->p, nc);
        b->cap = nc;
    }
    memcpy(b->p + b->len, d, n);
    b->len += n;
}
static void bb_u64(bbuf *b, uint64_t x) { uint8_t t[8]; u64le(t, x); bb_put(b, t, 8); }

/* Opening (proof.rs:29-42) serialized in field order */
static void emit_opening(bbuf *o, const trace_cols *tc, size_t c, const col_commit *cc, size_t row) {
    char label[64];
    label_of(c, tc->tau, label);
    size_t n = tc->n;
    size_t ch = row / COL_CHUNK, in = row - ch * COL_CHUNK;
    size_t s = ch * COL_CHUNK, e = s + COL_CHUNK < n ? s + COL_CHUNK : n;
    uint8_t *lv = (uint8_t *)malloc(32 * (e - s));
    chunk_leaves(tc, c, label, s, e, lv);           /* open_within_chunk (openings.rs:464-497) */
    mtree t;
    mtree_build(&t, lv, e - s);
    uint8_t sibs[64 * 32];
    size_t ns = mtree_open(&t, in, sibs);
    uint8_t v[8];
    u64le(v, COL(tc, c, row));
    bb_put(o, v, 8);                                  /* value_le */
    bb_u64(o, row);                                   /* index */
    bb_u64(o, ch);                                    /* chunk_index */
    bb_u64(o, in);                                    /* index_in_chunk */
    bb_put(o, mtree_root(&t), 32);                    /* chunk_root */
    bb_u64(o, ns);
    bb_put(o, sibs, 32 * ns);                         /* path_in_chunk */
    mtree_free(&t);
    free(lv);
    mtree ot;                                         /* outer tree (openings.rs:436-460) */
    mtree_build(&ot, cc->chunk_roots, cc->n_chunks);
    ns = mtree_open(&ot, ch, sibs);
    bb_u64(o, ns);
    bb_put(o, sibs, 32 * ns);                         /* path_to_chunk */
    mtree_free(&ot);
}

/* ========================================================================
 * Streaming LDE + DEEP — lde.rs:42-97
 * ====================================================================== */
static uint64_t *lde_deep(const uint64_t *base_vals, size_t n, unsigned blow_log2, uint64_t shift, uint64_t z) {
    unsigned base_log2 = 0;
    while (((size_t)1 << base_log2) < n) base_log2++;
    unsigned k = base_log2 + blow_log2;
    size_t N = (size_t)1 << k;
    uint64_t *coeffs = (uint64_t *)malloc(n * sizeof(uint64_t));
    memcpy(coeffs, base_vals, n * sizeof(uint64_t));
    ntt_core(coeffs, n, 1);                          /* interpolate_from_evals */
    uint64_t *y = (uint64_t *)malloc(N * sizeof(uint64_t));
    orc_coset_lde(coeffs, n, k, shift, y);           /* evaluate_on_coset_pow2 */
    free(coeffs);
    uint64_t w = gl_root_2exp(k);
    #pragma omp parallel for schedule(static) if (N >= 4096)
    for (size_t c0 = 0; c0 < N; c0 += 1024) {        /* lde.rs:80-93, chunks restart w^i */
        uint64_t wp = gl_pow(w, c0);
        for (size_t i = c0; i < N && i < c0 + 1024; i++) {
            uint64_t x = gl_mul(shift, wp);
            uint64_t d = gl_sub(x, z);
            y[i] = gl_mul(y[i], gl_inv(d));
            wp = gl_mul(wp, w);
        }
    }
    return y;
}

/* lde.rs:42-97 with the coset shift as a parameter (deep_coset_lde_stream
 * takes it from its caller; the prover passes 3, prover.rs:119) */
void orc_lde_deep_shift(const uint64_t *base_vals, size_t n, unsigned blow_log2, uint64_t shift, uint64_t z,
                        uint64_t *out) {
    uint64_t *y = lde_deep(base_vals, n, blow_log2, shift, z);
    memcpy(out, y, (n << blow_log2) * sizeof(uint64_t));
    free(y);
}

/* lde.rs:42-97 as a standalone entry (blowup 2^blow_log2, shift 3) */
void orc_lde_deep(const uint64_t *base_vals, size_t n, unsigned blow_log2, uint64_t z, uint64_t *out) {
    uint64_t *y = lde_deep(base_vals, n, blow_log2, 3, z);
    memcpy(out, y, (n << blow_log2) * sizeof(uint64_t));
    free(y);
}

/* ========================================================================
 * prove_v1 — prover.rs:61-462
 * ====================================================================== */
typedef struct {
    trace_cols tc;
    col_commit *cc;
    alphas_t al;
    uint64_t mask[4];
    uint64_t z;
    uint64_t *base_vals;
    uint64_t *lde;
    size_t N;
    unsigned k;
    orc_transcript tr;
} prove_state;

static int prove_front(const orc_blocks *b, const uint8_t mroot[32], prove_state *ps, char *err, size_t err_len) {
    int rc = build_cols(b, &ps->tc, err, err_len);  /* shape errors are reported here */
    if (rc) return rc;
    trace_cols *tc = &ps->tc;
    size_t n = tc->n;
    if (n == 0 || (n & (n - 1)) != 0) {
        snprintf(err, err_len, "n_base must be a power of two (got %zu)", n); /* lde.rs:51 */
        free(tc->col);
        return -3;
    }
    /* transcript prelude (prover.rs:67-70) */
    tr_init(&ps->tr, "sezkp-stark/v1");
    tr_absorb(&ps->tr, "manifest_root", mroot, 32);
    tr_absorb_u64(&ps->tr, "n", n);
    tr_absorb_u64(&ps->tr, "tau", tc->tau);
    /* column commitments (prover.rs:75-81) */
    ps->cc = (col_commit *)calloc(tc->ncols, sizeof(col_commit));
    #pragma omp parallel for schedule(dynamic)
    for (size_t c = 0; c < tc->ncols; c++) commit_column(tc, c, &ps->cc[c]);
    tr_absorb_u64(&ps->tr, "n_cols", tc->ncols);
    for (size_t c = 0; c < tc->ncols; c++) tr_absorb(&ps->tr, "col_root", ps->cc[c].root, 32);
    /* alphas (params.rs:82-92; prover.rs:85-98) */
    uint8_t ab[64];
    tr_challenge(&ps->tr, "alphas", ab, 64);
    uint64_t a[8];
    for (int i = 0; i < 8; i++) a[i] = gl_from_u64(rd64le(ab + 8 * i));
    ps->al.bool_flag = a[0]; ps->al.mv_domain = a[1]; ps->al.head_update = a[2];
    ps->al.head_bits_bool = a[3]; ps->al.head_reconstruct = a[4]; ps->al.slack_bits_bool = a[5];
    ps->al.slack_reconstruct = a[6]; ps->al.sym_bits_bool = a[7]; ps->al.sym_reconstruct = a[0];
    ps->al.boundary_first = a[2]; ps->al.boundary_last = a[2];
    /* masks (masking.rs:56-79) */
    tr_absorb(&ps->tr, "masks", (const uint8_t *)"masks", 5);
    tr_absorb_u64(&ps->tr, "n_masks", 1);
    tr_absorb_u64(&ps->tr, "deg", 4);
    for (int j = 0; j < 4; j++) {
        uint8_t mb[8];
        tr_challenge(&ps->tr, "mask_coeff", mb, 8);
        ps->mask[j] = gl_from_u64(rd64le(mb));
    }
    /* OOD point + coset nudge (prover.rs:119-135) */
    unsigned base_log2 = 0;
    while (((size_t)1 << base_log2) < n) base_log2++;
    ps->k = base_log2 + 3;
    ps->N = (size_t)1 << ps->k;
    uint8_t zb[8];
    tr_challenge(&ps->tr, "ood_point", zb, 8);
    uint64_t z = gl_from_u64(rd64le(zb));
    uint64_t shift_inv = gl_inv(3);
    for (;;) {
        uint64_t t = gl_mul(z, shift_inv);
        for (unsigned i = 0; i < ps->k; i++) t = gl_mul(t, t);
        if (t != 1) break;
        z = gl_add(z, 1);
    }
    ps->z = z;
    /* base evaluations C(i) + R(ω^i) (prover.rs:142-158) */
    uint64_t w_base = gl_root_2exp(base_log2);
    ps->base_vals = (uint64_t *)malloc(n * sizeof(uint64_t));
    #pragma omp parallel for schedule(static) if (n >= 4096)
    for (size_t c0 = 0; c0 < n; c0 += 1024) {  /* chunks restart w^i */
        uint64_t xp = gl_pow(w_base, c0);
        for (size_t i = c0; i < n && i < c0 + 1024; i++) {
            uint64_t comp = gl_add(compose_row(tc, i, &ps->al), compose_boundary(tc, i, &ps->al));
            uint64_t m = 0; /* eval_mask_at, Horner (masking.rs:86-92) */
            for (int j = 3; j >= 0; j--) m = gl_add(gl_mul(m, xp), ps->mask[j]);
            ps->base_vals[i] = gl_add(comp, gl_add(0, m));
            xp = gl_mul(xp, w_base);
        }
    }
    ps->lde = lde_deep(ps->base_vals, n, 3, 3, z);
    return 0;
}

static void free_state(prove_state *ps) {
    for (size_t c = 0; c < ps->tc.ncols; c++) free(ps->cc[c].chunk_roots);
    free(ps->cc);
    free(ps->tc.col);
    free(ps->base_vals);
    free(ps->lde);
}

/* Reference-faithful recomputation of one layer-0 pass: compose + INTT + coset
 * NTT + DEEP + N leaf hashes + Merkle levels (fri_stream.rs:267-349). */
static void faithful_layer0_pass(const prove_state *ps) {
    size_t n = ps->tc.n;
    uint64_t w_base = gl_root_2exp(ps->k - 3), xp = 1;
    uint64_t *bv = (uint64_t *)malloc(n * sizeof(uint64_t));
    for (size_t i = 0; i < n; i++) {
        uint64_t comp = gl_add(compose_row(&ps->tc, i, &ps->al), compose_boundary(&ps->tc, i, &ps->al));
        uint64_t m = 0;
        for (int j = 3; j >= 0; j--) m = gl_add(gl_mul(m, xp), ps->mask[j]);
        bv[i] = gl_add(comp, m);
        xp = gl_mul(xp, w_base);
    }
    uint64_t *y = lde_deep(bv, n, 3, 3, ps->z);
    slb s;
    slb_init(&s);
    for (size_t i = 0; i < ps->N; i++) { uint8_t h[32]; orc_hash_leaf_u64(y[i], h); slb_absorb_leaf(&s, h); }
    uint8_t r[32];
    slb_finalize(&s, r);
    free(y);
    free(bv);
}

static int prove_impl(const orc_blocks *b, const uint8_t mroot[32], int mode,
                      uint8_t **out, size_t *out_len, char *err, size_t err_len) {
    prove_state ps;
    memset(&ps, 0, sizeof(ps));
    int rc = prove_front(b, mroot, &ps, err, err_len);
    if (rc) return rc;
    trace_cols *tc = &ps.tc;
    size_t n = tc->n, N = ps.N, tau = tc->tau;
    unsigned k = ps.k;
    /* layer-0 root via StreamingLayerBuilder (prover.rs:139-189) */
    uint8_t *leaves0 = (uint8_t *)malloc(32 * N);
    #pragma omp parallel for schedule(static) if (N >= 4096)
    for (size_t i = 0; i < N; i++) orc_hash_leaf_u64(ps.lde[i], leaves0 + 32 * i);
    uint8_t *roots = (uint8_t *)malloc(32 * (k + 1));
    mtree t0;
    mtree_build(&t0, leaves0, N);
    if (mode == 1) {  /* the reference's streaming builder (fri_stream.rs:55-121) */
        slb s;
        slb_init(&s);
        for (size_t i = 0; i < N; i++) slb_absorb_leaf(&s, leaves0 + 32 * i);
        slb_finalize(&s, roots);
    } else {          /* compute-once: the same root from the stored tree (a
                       * power-of-two MerkleTree root equals the streaming
                       * builder's) */
        memcpy(roots, mtree_root(&t0), 32);
    }
    free(leaves0);
    tr_absorb(&ps.tr, "fri_layer_root", roots, 32);
    /* betas (prover.rs:192-198) */
    size_t n_folds = k;
    uint8_t *bb = (uint8_t *)malloc(8 * n_folds);
    tr_challenge(&ps.tr, "fri_betas", bb, 8 * n_folds);
    uint64_t *betas = (uint64_t *)malloc(8 * n_folds);
    for (size_t i = 0; i < n_folds; i++) betas[i] = gl_from_u64(rd64le(bb + 8 * i));
    free(bb);
    /* folds + layer trees (prover.rs:200-239); keep every layer for openings */
    uint64_t **layers = (uint64_t **)calloc(k + 1, sizeof(uint64_t *));
    mtree *trees = (mtree *)calloc(k + 1, sizeof(mtree));
    layers[0] = ps.lde;
    trees[0] = t0;
    size_t cur = N;
    for (size_t r = 0; r < n_folds; r++) {
        size_t half = cur / 2;
        layers[r + 1] = (uint64_t *)malloc(8 * half);
        #pragma omp parallel for schedule(static) if (half >= 4096)
        for (size_t i = 0; i < half; i++)
            layers[r + 1][i] = gl_add(layers[r][i], gl_mul(betas[r], layers[r][i + half]));
        cur = half;
        uint8_t *lv = (uint8_t *)malloc(32 * cur);
        #pragma omp parallel for schedule(static) if (cur >= 4096)
        for (size_t i = 0; i < cur; i++) orc_hash_leaf_u64(layers[r + 1][i], lv + 32 * i);
        mtree_build(&trees[r + 1], lv, cur);
        free(lv);
        memcpy(roots + 32 * (r + 1), mtree_root(&trees[r + 1]), 32);
        tr_absorb(&ps.tr, "fri_layer_root", roots + 32 * (r + 1), 32);
    }
    uint64_t final_val = layers[k][0];
    /* AIR row queries (prover.rs:248) */
    uint8_t qb[240];
    tr_challenge(&ps.tr, "row_queries", qb, 240);
    size_t rows[30];
    for (int i = 0; i < 30; i++) rows[i] = (size_t)(rd64le(qb + 8 * i) % (uint64_t)n);
    /* FRI queries (prover.rs:297) */
    tr_challenge(&ps.tr, "row_queries", qb, 240);
    size_t frows[30];
    for (int i = 0; i < 30; i++) frows[i] = (size_t)(rd64le(qb + 8 * i) % (uint64_t)N);

    if (mode == 1) {
        /* reference-faithful cost: 2 x 30 x k extra layer-0 passes, plus
         * per-open chunk rebuilds from row 0 (timing only; bytes identical) */
        for (int q = 0; q < 30; q++)
            for (int side = 0; side < 2; side++)
                for (unsigned lvl = 0; lvl < k; lvl++) faithful_layer0_pass(&ps);
    }

    /* serialize ProofV1 with bincode (proof.rs:80-98) */
    bbuf o = {0};
    bb_u64(&o, N);                                   /* domain_n */
    bb_u64(&o, tau);                                 /* tau */
    bb_u64(&o, tc->ncols);                           /* col_roots */
    for (size_t c = 0; c < tc->ncols; c++) {
        char label[64];
        label_of(c, tau, label);
        bb_u64(&o, strlen(label));
        bb_put(&o, label, strlen(label));
        bb_put(&o, ps.cc[c].root, 32);
    }
    bb_u64(&o, 30);                                  /* queries */
    for (int q = 0; q < 30; q++) {
        size_t row = rows[q], ip1 = (row + 1 < n) ? row + 1 : 0; /* next_wrap */
        bb_u64(&o, row);
        bb_u64(&o, tau);                             /* per_tape */
        for (size_t r = 0; r < tau; r++) {
            emit_opening(&o, tc, 3 + K_MV * tau + r, &ps.cc[3 + K_MV * tau + r], row);
            emit_opening(&o, tc, 3 + K_MV * tau + r, &ps.cc[3 + K_MV * tau + r], ip1);
            emit_opening(&o, tc, 3 + K_WFLAG * tau + r, &ps.cc[3 + K_WFLAG * tau + r], row);
            emit_opening(&o, tc, 3 + K_WSYM * tau + r, &ps.cc[3 + K_WSYM * tau + r], row);
            emit_opening(&o, tc, 3 + K_HEAD * tau + r, &ps.cc[3 + K_HEAD * tau + r], row);
            emit_opening(&o, tc, 3 + K_HEAD * tau + r, &ps.cc[3 + K_HEAD * tau + r], ip1);
            emit_opening(&o, tc, 3 + K_WINLEN * tau + r, &ps.cc[3 + K_WINLEN * tau + r], row);
            emit_opening(&o, tc, 3 + K_INOFF * tau + r, &ps.cc[3 + K_INOFF * tau + r], row);
            emit_opening(&o, tc, 3 + K_OUTOFF * tau + r, &ps.cc[3 + K_OUTOFF * tau + r], row);
        }
        emit_opening(&o, tc, 1, &ps.cc[1], row);     /* is_first */
        emit_opening(&o, tc, 2, &ps.cc[2], row);     /* is_last */
        emit_opening(&o, tc, 0, &ps.cc[0], row);     /* input_mv */
    }
    bb_u64(&o, k + 1);                               /* fri_roots */
    bb_put(&o, roots, 32 * (k + 1));
    bb_u64(&o, 30);                                  /* fri_queries */
    uint8_t sibs[64 * 32];
    for (int q = 0; q < 30; q++) {
        size_t pos[64];
        pos[0] = frows[q];
        size_t len = N;
        for (unsigned r = 0; r < k; r++) { pos[r + 1] = pos[r] % (len / 2); len /= 2; }
        bb_u64(&o, k + 1);                           /* positions */
        for (unsigned r = 0; r <= k; r++) bb_u64(&o, pos[r]);
        bb_u64(&o, k);                               /* pairs */
        len = N;
        for (unsigned r = 0; r < k; r++) {
            size_t half = len / 2, i = pos[r], j = i ^ half;
            uint8_t v[8];
            u64le(v, layers[r][i]);
            bb_put(&o, v, 8);
            size_t ns = mtree_open(&trees[r], i, sibs);
            bb_u64(&o, ns);
            bb_put(&o, sibs, 32 * ns);
            u64le(v, layers[r][j]);
            bb_put(&o, v, 8);
            ns = mtree_open(&trees[r], j, sibs);
            bb_u64(&o, ns);
            bb_put(&o, sibs, 32 * ns);
            len = half;
        }
    }
    uint8_t fv[8];
    u64le(fv, final_val);
    bb_put(&o, fv, 8);                               /* fri_final_value_le */
    bb_put(&o, mroot, 32);                           /* manifest_root */

    for (unsigned r = 0; r <= k; r++) { mtree_free(&trees[r]); if (r) free(layers[r]); }
    free(trees);
    free(layers);
    free(betas);
    free(roots);
    free_state(&ps);
    *out = o.p;
    *out_len = o.len;
    return 0;
}

int orc_prove_v1(const orc_blocks *b, const uint8_t manifest_root[32], int mode,
                 uint8_t **out, size_t *out_len, char *err, size_t err_len) {
    if (err && err_len) err[0] = 0;
    return prove_impl(b, manifest_root, mode, out, out_len, err, err_len);
}

int orc_prove_v1_debug(const orc_blocks *b, const uint8_t mroot[32], uint8_t *col_roots,
                       uint64_t *base_evals, uint64_t *lde_vals, uint8_t *fri_roots, char *err, size_t err_len) {
    prove_state ps;
    memset(&ps, 0, sizeof(ps));
    int rc = prove_front(b, mroot, &ps, err, err_len);
    if (rc) return rc;
    if (col_roots)
        for (size_t c = 0; c < ps.tc.ncols; c++) memcpy(col_roots + 32 * c, ps.cc[c].root, 32);
    if (base_evals) memcpy(base_evals, ps.base_vals, 8 * ps.tc.n);
    if (lde_vals) memcpy(lde_vals, ps.lde, 8 * ps.N);
    if (fri_roots) {
        uint8_t *lv = (uint8_t *)malloc(32 * ps.N);
        for (size_t i = 0; i < ps.N; i++) orc_hash_leaf_u64(ps.lde[i], lv + 32 * i);
        orc_merkle_root(lv, ps.N, fri_roots);
        free(lv);
    }
    free_state(&ps);
    return 0;
}

void orc_free(void *p) { free(p); }
#ifdef _OPENMP
#include <omp.h>
int orc_set_threads(int n) { if (n > 0) omp_set_num_threads(n); return omp_get_max_threads(); }
#else
int orc_set_threads(int n) { (void)n; return 1; }
#endif

double orc_time_lde_pass(const orc_blocks *b, const uint8_t mroot[32]) {
    prove_state ps;
    char err[256];
    memset(&ps, 0, sizeof(ps));
    if (prove_front(b, mroot, &ps, err, sizeof err)) return -1.0;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    faithful_layer0_pass(&ps);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free_state(&ps);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
