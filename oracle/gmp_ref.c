/*
 * gmp_ref.c -- TEST INFRASTRUCTURE ONLY (parity cross-check + CPU baseline).
 *
 * The reference's Paillier path is Rust over rug 1.20.1, which wraps GMP
 * (rust/fate_utils/Cargo.toml:8).  It cannot be built here (no cargo), so this file
 * issues the SAME sequence of GMP calls rug makes for each operation, element by
 * element, with no FFI overhead:
 *   encrypt  crates/paillier/src/lib.rs:104-121  (m*n+1 tdiv n^2; random_below(n-1)+1;
 *            mpz_powm(r, n, n^2); mul; tdiv_r)
 *   decrypt  crates/paillier/src/lib.rs:163-176  (2x h_function: powm, sub 1, tdiv_q,
 *            mul, tdiv_r; CRT with tdiv_r; +n if negative)
 *   add      crates/paillier/src/lib.rs:35-37    (mpz_mul + mpz_tdiv_r)
 *   ct x pt  fixedpoint_paillier/src/lib.rs:334-349 (mpz_powm by the significand; a
 *            negative one inverts the base first, mpz_invert, as GMP's powm does)
 *   iupdate  fixedpoint_paillier/src/lib.rs:724-735 (a sequential Ciphertext::add of each
 *            term into its slot, :301-333, decrese_exp_to's mpz_powm by 16^gap included)
 * The image ships libgmp.so.10 (6.2.1) without gmp.h, so the few entry points used are
 * declared below against GMP's documented, stable ABI (__gmpz_* symbols, mpz_t layout).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <time.h>

typedef unsigned long mp_limb_t;
typedef struct { int _mp_alloc; int _mp_size; mp_limb_t* _mp_d; } mpz_struct;
typedef mpz_struct mpz_t[1];
typedef struct { mpz_struct seed; int alg; void* algdata; } randstate_struct;
typedef randstate_struct randstate_t[1];

extern void __gmpz_init(mpz_struct*);
extern void __gmpz_clear(mpz_struct*);
extern int __gmpz_set_str(mpz_struct*, const char*, int);
extern char* __gmpz_get_str(char*, int, const mpz_struct*);
extern void __gmpz_set(mpz_struct*, const mpz_struct*);
extern void __gmpz_set_ui(mpz_struct*, unsigned long);
extern void __gmpz_powm(mpz_struct*, const mpz_struct*, const mpz_struct*, const mpz_struct*);
extern void __gmpz_mul(mpz_struct*, const mpz_struct*, const mpz_struct*);
extern void __gmpz_add(mpz_struct*, const mpz_struct*, const mpz_struct*);
extern void __gmpz_sub(mpz_struct*, const mpz_struct*, const mpz_struct*);
extern void __gmpz_add_ui(mpz_struct*, const mpz_struct*, unsigned long);
extern void __gmpz_sub_ui(mpz_struct*, const mpz_struct*, unsigned long);
extern void __gmpz_tdiv_r(mpz_struct*, const mpz_struct*, const mpz_struct*);
extern void __gmpz_tdiv_q(mpz_struct*, const mpz_struct*, const mpz_struct*);
extern int __gmpz_invert(mpz_struct*, const mpz_struct*, const mpz_struct*);
extern void __gmpz_urandomm(mpz_struct*, randstate_struct*, const mpz_struct*);
extern void __gmpz_mul_2exp(mpz_struct*, const mpz_struct*, unsigned long);
extern void __gmp_randinit_default(randstate_struct*);
extern void __gmp_randseed_ui(randstate_struct*, unsigned long);
extern void __gmp_randclear(randstate_struct*);
extern void (*__gmp_free_func)(void*, size_t);

#define SGN(z) (((z)->_mp_size > 0) - ((z)->_mp_size < 0))

typedef struct {
  mpz_t n, ns, nm1, p, q, ps, qs, pm1, qm1, pinv, hp, hq;
  int has_sk;
} gref_ctx;

static void h_function(mpz_struct* out, const mpz_struct* c, const mpz_struct* p, const mpz_struct* p1,
                       const mpz_struct* ps, const mpz_struct* hp, mpz_struct* t) {
  /* ((c.pow_mod(p-1, ps) - 1) / p * hp) % p   (paillier/src/lib.rs:174-176) */
  __gmpz_powm(t, c, p1, ps);
  __gmpz_sub_ui(t, t, 1);
  __gmpz_tdiv_q(t, t, p);
  __gmpz_mul(t, t, hp);
  __gmpz_tdiv_r(out, t, p);
}

gref_ctx* gref_new(const char* n_hex, const char* p_hex, const char* q_hex) {
  gref_ctx* c = (gref_ctx*)calloc(1, sizeof(gref_ctx));
  mpz_struct* all[] = {c->n, c->ns, c->nm1, c->p, c->q, c->ps, c->qs, c->pm1, c->qm1, c->pinv, c->hp, c->hq};
  for (unsigned i = 0; i < sizeof(all) / sizeof(all[0]); ++i) __gmpz_init(all[i]);
  __gmpz_set_str(c->n, n_hex, 16);
  __gmpz_mul(c->ns, c->n, c->n);
  __gmpz_sub_ui(c->nm1, c->n, 1);
  if (p_hex && q_hex) {
    c->has_sk = 1;
    __gmpz_set_str(c->p, p_hex, 16);
    __gmpz_set_str(c->q, q_hex, 16);
    __gmpz_mul(c->ps, c->p, c->p);
    __gmpz_mul(c->qs, c->q, c->q);
    __gmpz_sub_ui(c->pm1, c->p, 1);
    __gmpz_sub_ui(c->qm1, c->q, 1);
    __gmpz_invert(c->pinv, c->p, c->q);
    /* SK::new (paillier/src/lib.rs:131-137) */
    mpz_t g, t;
    __gmpz_init(g); __gmpz_init(t);
    __gmpz_add_ui(g, c->n, 1);
    __gmpz_powm(t, g, c->pm1, c->ps); __gmpz_sub_ui(t, t, 1); __gmpz_tdiv_q(t, t, c->p); __gmpz_invert(c->hp, t, c->p);
    __gmpz_powm(t, g, c->qm1, c->qs); __gmpz_sub_ui(t, t, 1); __gmpz_tdiv_q(t, t, c->q); __gmpz_invert(c->hq, t, c->q);
    __gmpz_clear(g); __gmpz_clear(t);
  }
  return c;
}

void gref_free(gref_ctx* c) {
  if (!c) return;
  mpz_struct* all[] = {c->n, c->ns, c->nm1, c->p, c->q, c->ps, c->qs, c->pm1, c->qm1, c->pinv, c->hp, c->hq};
  for (unsigned i = 0; i < sizeof(all) / sizeof(all[0]); ++i) __gmpz_clear(all[i]);
  free(c);
}

static void out_str(char* out, size_t cap, const mpz_struct* v) {
  char* s = __gmpz_get_str(NULL, 16, v);
  size_t l = strlen(s);
  if (l + 1 <= cap) memcpy(out, s, l + 1); else out[0] = 0;
  __gmp_free_func(s, l + 1);
}

/* encrypt (paillier/src/lib.rs:104-121) with injected r (hex) */
int gref_encrypt(gref_ctx* c, const char* m_hex, const char* r_hex, int obf, char* out, size_t cap) {
  mpz_t m, nude, t, r;
  __gmpz_init(m); __gmpz_init(nude); __gmpz_init(t); __gmpz_init(r);
  __gmpz_set_str(m, m_hex, 16);
  mpz_t q4; __gmpz_init(q4);
  __gmpz_set(q4, c->n);
  {
    /* n >> 2 */
    mpz_t four; __gmpz_init(four); __gmpz_set_ui(four, 4); __gmpz_tdiv_q(q4, c->n, four); __gmpz_clear(four);
  }
  /* compare m > n>>2 via subtraction sign */
  __gmpz_sub(t, m, q4);
  if (SGN(t) > 0) {
    __gmpz_sub(t, c->n, m);
    __gmpz_mul(t, c->n, t);
    __gmpz_add_ui(t, t, 1);
    __gmpz_tdiv_r(t, t, c->ns);
    __gmpz_invert(nude, t, c->ns);
  } else {
    __gmpz_mul(t, m, c->n);
    __gmpz_add_ui(t, t, 1);
    __gmpz_tdiv_r(nude, t, c->ns);
  }
  if (obf) {
    __gmpz_set_str(r, r_hex, 16);
    __gmpz_powm(t, r, c->n, c->ns);
    __gmpz_mul(t, nude, t);
    __gmpz_tdiv_r(nude, t, c->ns);
  }
  out_str(out, cap, nude);
  __gmpz_clear(m); __gmpz_clear(nude); __gmpz_clear(t); __gmpz_clear(r); __gmpz_clear(q4);
  return 0;
}

int gref_decrypt(gref_ctx* c, const char* c_hex, char* out, size_t cap) {
  if (!c->has_sk) return -1;
  mpz_t ct, dp, dq, t, o;
  __gmpz_init(ct); __gmpz_init(dp); __gmpz_init(dq); __gmpz_init(t); __gmpz_init(o);
  __gmpz_set_str(ct, c_hex, 16);
  h_function(dp, ct, c->p, c->pm1, c->ps, c->hp, t);
  h_function(dq, ct, c->q, c->qm1, c->qs, c->hq, t);
  __gmpz_sub(o, dq, dp);
  __gmpz_mul(o, o, c->pinv);
  __gmpz_tdiv_r(o, o, c->q);
  __gmpz_mul(o, o, c->p);
  __gmpz_add(o, o, dp);
  if (SGN(o) < 0) __gmpz_add(o, o, c->n);
  out_str(out, cap, o);
  __gmpz_clear(ct); __gmpz_clear(dp); __gmpz_clear(dq); __gmpz_clear(t); __gmpz_clear(o);
  return 0;
}

int gref_add_ct(gref_ctx* c, const char* a_hex, const char* b_hex, char* out, size_t cap) {
  mpz_t a, b;
  __gmpz_init(a); __gmpz_init(b);
  __gmpz_set_str(a, a_hex, 16); __gmpz_set_str(b, b_hex, 16);
  __gmpz_mul(a, a, b);
  __gmpz_tdiv_r(a, a, c->ns);
  out_str(out, cap, a);
  __gmpz_clear(a); __gmpz_clear(b);
  return 0;
}

int gref_powm(const char* b_hex, const char* e_hex, const char* m_hex, char* out, size_t cap) {
  mpz_t b, e, m, r;
  __gmpz_init(b); __gmpz_init(e); __gmpz_init(m); __gmpz_init(r);
  __gmpz_set_str(b, b_hex, 16); __gmpz_set_str(e, e_hex, 16); __gmpz_set_str(m, m_hex, 16);
  __gmpz_powm(r, b, e, m);
  out_str(out, cap, r);
  __gmpz_clear(b); __gmpz_clear(e); __gmpz_clear(m); __gmpz_clear(r);
  return 0;
}

int gref_tdiv_r(const char* a_hex, const char* m_hex, char* out, size_t cap) {
  mpz_t a, m;
  __gmpz_init(a); __gmpz_init(m);
  __gmpz_set_str(a, a_hex, 16); __gmpz_set_str(m, m_hex, 16);
  __gmpz_tdiv_r(a, a, m);
  out_str(out, cap, a);
  __gmpz_clear(a); __gmpz_clear(m);
  return 0;
}

/* ---------------- bulk vector checkers (binary, threaded) ----------------
 * Every vector crosses this interface as the reference's signed integers: element i is the
 * magnitude in L little-endian uint32 words at w[i*L], a negative flag neg[i] and the base-16
 * exponent exp[i] (the device's fphe_export_signed layout).  The ops are the reference's
 * sequential loops, element by element, on libgmp (the library rug wraps):
 *   gref_fold     iupdate / intervals_sum / matmul's add_assign loop (lib.rs:724-791, 861-908):
 *                 acc[slot[k]] = Ciphertext::add(acc[slot[k]], src[term[k]]) for k ascending
 *   gref_mul      Ciphertext::mul (lib.rs:334-349), both branches and the panic
 *   gref_squeeze  CiphertextVector::pack_squeeze (lib.rs:439-450)
 *   gref_cumsum   CiphertextVector::chunking_cumsum_with_step (lib.rs:760-771)
 * Slots (fold) or elements (mul) are split over `threads` pthreads; each thread owns its slots
 * outright, so the per-slot term order is the reference's. */
extern void __gmpz_import(mpz_struct*, size_t, int, size_t, int, size_t, const void*);
extern void* __gmpz_export(void*, size_t*, int, size_t, int, size_t, const mpz_struct*);
extern void __gmpz_neg(mpz_struct*, const mpz_struct*);
extern int __gmpz_cmp(const mpz_struct*, const mpz_struct*);
extern int __gmpz_cmp_ui(const mpz_struct*, unsigned long);
extern void __gmpz_tdiv_q_2exp(mpz_struct*, const mpz_struct*, unsigned long);

static void ld_ct(mpz_struct* z, const uint32_t* w, int L, int neg) {
  __gmpz_import(z, (size_t)L, -1, 4, 0, 0, w);
  if (neg) __gmpz_neg(z, z);
}
/* returns -1 when |z| needs more than L words (never for values < n^2 at the key's L) */
static int st_ct(uint32_t* w, int L, uint8_t* neg, const mpz_struct* z) {
  size_t cnt = 0;
  memset(w, 0, 4u * (size_t)L);
  if (SGN(z) != 0) {
    const size_t bits = (size_t)(z->_mp_size < 0 ? -z->_mp_size : z->_mp_size) * 64u;
    if (bits > 32u * (size_t)L + 64u) return -1;
    uint32_t tmp[4096 / 32 * 2 + 4];
    __gmpz_export(tmp, &cnt, -1, 4, 0, 0, z);
    if (cnt > (size_t)L) return -1;
    memcpy(w, tmp, 4u * cnt);
  }
  *neg = SGN(z) < 0;
  return 0;
}
static int is_literal_one(const mpz_struct* z) { return z->_mp_size == 1 && z->_mp_d[0] == 1; }
static void fp_add_into(gref_ctx* c, mpz_struct* acc, int* ae, const mpz_struct* tc, int te, mpz_struct* t,
                        mpz_struct* e16);

typedef struct {
  gref_ctx* c; int L; int tid, threads; int rc;
  const uint32_t* sw; const uint8_t* sn; const int32_t* se;
  const int64_t* term; const int64_t* slot; long nterms; long nslots;
  uint32_t* aw; uint8_t* an; int32_t* ae;
} fold_job;

static void* fold_worker(void* arg) {
  fold_job* j = (fold_job*)arg;
  const long nown = (j->nslots - j->tid + j->threads - 1) / j->threads;
  mpz_struct* acc = (mpz_struct*)calloc(nown > 0 ? nown : 1, sizeof(mpz_struct));
  int* ae = (int*)calloc(nown > 0 ? nown : 1, sizeof(int));
  mpz_t term, t, e16;
  __gmpz_init(term); __gmpz_init(t); __gmpz_init(e16);
  for (long s = j->tid, k = 0; s < j->nslots; s += j->threads, ++k) {
    __gmpz_init(&acc[k]);
    ld_ct(&acc[k], j->aw + (size_t)s * j->L, j->L, j->an[s]);
    ae[k] = j->ae[s];
  }
  for (long k = 0; k < j->nterms; ++k) {
    const long s = (long)j->slot[k];
    if (s % j->threads != j->tid) continue;
    const long i = (long)j->term[k];
    ld_ct(term, j->sw + (size_t)i * j->L, j->L, j->sn[i]);
    mpz_struct* a = &acc[s / j->threads];
    int* e = &ae[s / j->threads];
    /* add(a, b): a literal 1 returns b, then b literal 1 returns a (lib.rs:303-308) */
    if (!is_literal_one(a) && is_literal_one(term)) continue;
    fp_add_into(j->c, a, e, term, j->se[i], t, e16);
  }
  for (long s = j->tid, k = 0; s < j->nslots; s += j->threads, ++k) {
    if (st_ct(j->aw + (size_t)s * j->L, j->L, j->an + s, &acc[k])) j->rc = -1;
    j->ae[s] = ae[k];
    __gmpz_clear(&acc[k]);
  }
  free(acc); free(ae);
  __gmpz_clear(term); __gmpz_clear(t); __gmpz_clear(e16);
  return NULL;
}

/* acc (nslots elements, in/out: the target vector's current state) += the listed terms */
int gref_fold(gref_ctx* c, int L, const uint32_t* sw, const uint8_t* sn, const int32_t* se, const int64_t* term,
              const int64_t* slot, long nterms, uint32_t* aw, uint8_t* an, int32_t* ae, long nslots, int threads) {
  if (threads < 1) threads = 1;
  pthread_t th[64];
  fold_job jobs[64];
  if (threads > 64) threads = 64;
  for (int t = 0; t < threads; ++t) {
    fold_job j = {c, L, t, threads, 0, sw, sn, se, term, slot, nterms, nslots, aw, an, ae};
    jobs[t] = j;
    pthread_create(&th[t], NULL, fold_worker, &jobs[t]);
  }
  int rc = 0;
  for (int t = 0; t < threads; ++t) { pthread_join(th[t], NULL); rc |= jobs[t].rc; }
  return rc;
}

typedef struct {
  gref_ctx* c; int L, Lp; int tid, threads; int rc;
  const uint32_t* sw; const uint8_t* sn; const int32_t* se;
  const uint32_t* pw; const uint8_t* pn; const int32_t* pe; long n;
  uint32_t* ow; uint8_t* on; int32_t* oe;
} mul_job;

static void* mul_worker(void* arg) {
  mul_job* j = (mul_job*)arg;
  mpz_t ct, b, r, t, maxint, big;
  __gmpz_init(ct); __gmpz_init(b); __gmpz_init(r); __gmpz_init(t); __gmpz_init(maxint); __gmpz_init(big);
  __gmpz_tdiv_q_2exp(maxint, j->c->n, 1);   /* max_int = n / 2 (lib.rs:408-413) */
  __gmpz_sub(big, j->c->n, maxint);         /* n - max_int */
  for (long i = j->tid; i < j->n; i += j->threads) {
    ld_ct(ct, j->sw + (size_t)i * j->L, j->L, j->sn[i]);
    ld_ct(b, j->pw + (size_t)i * j->Lp, j->Lp, j->pn[i]);
    if (__gmpz_cmp(big, b) <= 0) {          /* large plaintext: invert(c)^(n - b) */
      if (!__gmpz_invert(t, ct, j->c->ns)) { j->rc = -2; continue; }
      __gmpz_sub(r, j->c->n, b);
      __gmpz_powm(r, t, r, j->c->ns);
    } else if (__gmpz_cmp(b, maxint) <= 0) { /* c^b (a negative b inverts inside powm) */
      if (SGN(b) < 0 && !__gmpz_invert(t, ct, j->c->ns)) { j->rc = -2; continue; }
      __gmpz_powm(r, ct, b, j->c->ns);
    } else {
      j->rc = -3;                           /* panic!("invalid plaintext") */
      continue;
    }
    if (st_ct(j->ow + (size_t)i * j->L, j->L, j->on + i, r)) j->rc = -1;
    j->oe[i] = j->se[i] + j->pe[i];
  }
  __gmpz_clear(ct); __gmpz_clear(b); __gmpz_clear(r); __gmpz_clear(t); __gmpz_clear(maxint); __gmpz_clear(big);
  return NULL;
}

/* out[i] = Ciphertext::mul(src[i], pt[i]); pt significands signed (Lp words + negative flag) */
int gref_mul(gref_ctx* c, int L, const uint32_t* sw, const uint8_t* sn, const int32_t* se, int Lp, const uint32_t* pw,
             const uint8_t* pn, const int32_t* pe, long n, uint32_t* ow, uint8_t* on, int32_t* oe, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 64) threads = 64;
  pthread_t th[64];
  mul_job jobs[64];
  for (int t = 0; t < threads; ++t) {
    mul_job j = {c, L, Lp, t, threads, 0, sw, sn, se, pw, pn, pe, n, ow, on, oe};
    jobs[t] = j;
    pthread_create(&th[t], NULL, mul_worker, &jobs[t]);
  }
  int rc = 0;
  for (int t = 0; t < threads; ++t) { pthread_join(th[t], NULL); if (jobs[t].rc) rc = jobs[t].rc; }
  return rc;
}

/* pack_squeeze: per chunk of pack_num, acc = x0; acc = powm(acc, 2^shift) * y tdiv n^2 */
int gref_squeeze(gref_ctx* c, int L, const uint32_t* sw, const uint8_t* sn, long n, int pack_num,
                 unsigned long shift_bit, uint32_t* ow, uint8_t* on, int32_t* oe) {
  mpz_t acc, y, base, t;
  __gmpz_init(acc); __gmpz_init(y); __gmpz_init(base); __gmpz_init(t);
  __gmpz_set_ui(base, 1);
  __gmpz_mul_2exp(base, base, shift_bit);
  int rc = 0;
  for (long h = 0, o = 0; h < n; h += pack_num, ++o) {
    ld_ct(acc, sw + (size_t)h * L, L, sn[h]);
    for (long k = h + 1; k < h + pack_num && k < n; ++k) {
      __gmpz_powm(acc, acc, base, c->ns);
      ld_ct(y, sw + (size_t)k * L, L, sn[k]);
      __gmpz_mul(t, acc, y);
      __gmpz_tdiv_r(acc, t, c->ns);
    }
    if (st_ct(ow + (size_t)o * L, L, on + o, acc)) rc = -1;
    oe[o] = 0;
  }
  __gmpz_clear(acc); __gmpz_clear(y); __gmpz_clear(base); __gmpz_clear(t);
  return rc;
}

/* chunking_cumsum_with_step in place: data[i+j] = add(data[i+j], data[i+j-step]), j ascending */
int gref_cumsum(gref_ctx* c, int L, uint32_t* w, uint8_t* ng, int32_t* ex, long n, const int64_t* chunks,
                long nchunks, long step) {
  mpz_t a, b, t, e16;
  __gmpz_init(a); __gmpz_init(b); __gmpz_init(t); __gmpz_init(e16);
  int rc = 0;
  long base = 0;
  for (long ci = 0; ci < nchunks; ++ci) {
    for (long j = step; j < chunks[ci]; ++j) {
      const long d = base + j, s = d - step;
      if (d >= n) { rc = -4; break; }
      ld_ct(a, w + (size_t)d * L, L, ng[d]);
      ld_ct(b, w + (size_t)s * L, L, ng[s]);
      int ea = ex[d];
      if (!is_literal_one(a) && is_literal_one(b)) continue;
      fp_add_into(c, a, &ea, b, ex[s], t, e16);
      if (st_ct(w + (size_t)d * L, L, ng + d, a)) rc = -1;
      ex[d] = ea;
    }
    base += chunks[ci];
  }
  __gmpz_clear(a); __gmpz_clear(b); __gmpz_clear(t); __gmpz_clear(e16);
  return rc;
}

/* ---------------- timed CPU baseline (same call sequence, per element) ---------------- */
typedef struct {
  gref_ctx* c;
  long count;
  unsigned long seed;
  int op;  /* 0 encrypt(obfuscated), 1 decrypt, 2 add (aligned), 3 add (Hetero-LR exponent gaps),
              4 ct x pt (float32 weights in [-1, 2)), 5 iupdate (SecureBoost-shaped g, h terms) */
  double secs;
} job_t;

/* xorshift64* and a standard normal (Box-Muller) for the SecureBoost-shaped inputs */
static double urand(unsigned long* s) {
  *s ^= *s >> 12; *s ^= *s << 25; *s ^= *s >> 27;
  return (double)((*s * 2685821657736338717ull) >> 11) * (1.0 / 9007199254740992.0);
}
static double nrand(unsigned long* s) {
  const double u = urand(s) + 1e-300, v = urand(s);
  return sqrt(-2.0 * log(u)) * cos(6.283185307179586 * v);
}
/* Coder::encode_f64 (fixedpoint_paillier/src/lib.rs:148-168) of a float32 value: base-16
   exponent floor((frexp_e - 53) / 4) and the signed 53-bit significand x * 16^-exp (exact) */
static int encode_exp(double x) {
  int e;
  if (x == 0.0) return -14;
  (void)frexp(x, &e);
  const int d = e - 53;
  return d >= 0 ? d / 4 : -((-d + 3) / 4);
}

/* Ciphertext::add of `t` (exp te) into the slot (acc, ae): the literal-1 rule, the exponent
   alignment of the higher operand by mpz_powm(x, 16^gap, n^2), then add_ct */
static void fp_add_into(gref_ctx* c, mpz_struct* acc, int* ae, const mpz_struct* tc, int te, mpz_struct* t,
                        mpz_struct* e16) {
  if (acc->_mp_size == 1 && acc->_mp_d[0] == 1) {  /* literal 1: the slot becomes the term */
    __gmpz_set(acc, tc);
    *ae = te;
    return;
  }
  if (*ae > te) {
    __gmpz_set_ui(e16, 1);
    __gmpz_mul_2exp(e16, e16, 4u * (unsigned)(*ae - te));
    __gmpz_powm(acc, acc, e16, c->ns);
    __gmpz_mul(t, acc, tc);
    *ae = te;
  } else if (*ae < te) {
    __gmpz_set_ui(e16, 1);
    __gmpz_mul_2exp(e16, e16, 4u * (unsigned)(te - *ae));
    __gmpz_powm(t, tc, e16, c->ns);
    __gmpz_mul(t, acc, t);
  } else {
    __gmpz_mul(t, acc, tc);
  }
  __gmpz_tdiv_r(acc, t, c->ns);
}

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void* run_job(void* arg) {
  job_t* j = (job_t*)arg;
  gref_ctx* c = j->c;
  randstate_t rs;
  __gmp_randinit_default(rs);
  __gmp_randseed_ui(rs, j->seed);
  mpz_t m, nude, r, t, acc, dp, dq, o;
  __gmpz_init(m); __gmpz_init(nude); __gmpz_init(r); __gmpz_init(t); __gmpz_init(acc);
  __gmpz_init(dp); __gmpz_init(dq); __gmpz_init(o);
  /* a realistic ciphertext / operands */
  __gmpz_urandomm(acc, rs, c->ns);
  __gmpz_urandomm(o, rs, c->ns);
  /* iupdate: 4 features x 32 bins x (g, h) slots (the bench's histogram shape), literal 1s at
     first, and a pool of 64 source ciphertexts standing for the encrypted g and h */
  enum { kSlots = 256, kPool = 64 };
  mpz_struct* slot = NULL;
  int* sexp = NULL;
  mpz_struct* pool = NULL;
  unsigned long xs = j->seed * 0x9E3779B97F4A7C15ull + 1;
  if (j->op == 5) {
    slot = (mpz_struct*)calloc(kSlots, sizeof(mpz_struct));
    sexp = (int*)calloc(kSlots, sizeof(int));
    pool = (mpz_struct*)calloc(kPool, sizeof(mpz_struct));
    for (int k = 0; k < kSlots; ++k) { __gmpz_init(&slot[k]); __gmpz_set_ui(&slot[k], 1); }
    for (int k = 0; k < kPool; ++k) { __gmpz_init(&pool[k]); __gmpz_urandomm(&pool[k], rs, c->ns); }
  }
  double t0 = now_s();
  for (long i = 0; i < j->count; ++i) {
    if (j->op == 0) {
      /* m = float significand (~56 bits) */
      __gmpz_set_ui(m, (unsigned long)(0x00F0000000000000ull | (unsigned long)i));
      __gmpz_mul(t, m, c->n);
      __gmpz_add_ui(t, t, 1);
      __gmpz_tdiv_r(nude, t, c->ns);
      __gmpz_urandomm(r, rs, c->nm1);  /* gen_positive_integer: random_below(n-1) + 1 */
      __gmpz_add_ui(r, r, 1);
      __gmpz_powm(r, r, c->n, c->ns);
      __gmpz_mul(t, nude, r);
      __gmpz_tdiv_r(nude, t, c->ns);
    } else if (j->op == 1) {
      h_function(dp, acc, c->p, c->pm1, c->ps, c->hp, t);
      h_function(dq, acc, c->q, c->qm1, c->qs, c->hq, t);
      __gmpz_sub(nude, dq, dp);
      __gmpz_mul(nude, nude, c->pinv);
      __gmpz_tdiv_r(nude, nude, c->q);
      __gmpz_mul(nude, nude, c->p);
      __gmpz_add(nude, nude, dp);
      if (SGN(nude) < 0) __gmpz_add(nude, nude, c->n);
    } else if (j->op == 2) {
      __gmpz_mul(t, acc, o);
      __gmpz_tdiv_r(acc, t, c->ns);
    } else if (j->op == 4) {
      /* Ciphertext::mul by an encoded float32 weight w in [-1, 2) (encode_f32 widens to f64:
         a <= 56-bit significand whose low 29 bits are zero); w < 0 (a third): GMP powm with a
         negative exponent inverts the base first (math/src/rug/mod.rs:30-35) */
      const double wv = urand(&xs) * 3.0 - 1.0;
      const float wf = (float)wv;
      const int ex = encode_exp((double)wf);
      const double mag = ldexp(fabs((double)wf), -4 * ex);
      __gmpz_set_ui(m, (unsigned long)mag);
      if (wf < 0) {
        __gmpz_invert(r, acc, c->ns);
        __gmpz_powm(nude, r, m, c->ns);
      } else {
        __gmpz_powm(nude, acc, m, c->ns);
      }
    } else if (j->op == 5) {
      /* iupdate: one scatter-add of a SecureBoost-shaped term (g = p - y or h = p (1 - p),
         p = sigmoid(N(0, 1)), encoded float32 exponents) into a random slot */
      const double pv = 1.0 / (1.0 + exp(-nrand(&xs)));
      const int hterm = (int)(i & 1);
      const double v = hterm ? pv * (1.0 - pv) : pv - (urand(&xs) < 0.5 ? 1.0 : 0.0);
      const int te = encode_exp((double)(float)v);
      const int k = (int)(urand(&xs) * (kSlots / 2)) * 2 + hterm;
      fp_add_into(c, &slot[k], &sexp[k], &pool[i % kPool], te, t, m);
    } else {
      /* Ciphertext::add with exponent alignment (fixedpoint_paillier/src/lib.rs:301-333):
         decrese_exp_to (:250-258) raises the higher-exp operand to 16^gap through mul_pt
         (mpz_powm), then add_ct (paillier/src/lib.rs:35-37).  Gaps drawn as measured on the
         bench's Hetero-LR-shaped adds (profiles/r01f_add_leg.txt): 0 for 37%, 1 for 58%,
         2 for 5% of the elements. */
      const unsigned g = (unsigned)(i % 100);
      const unsigned gap = g < 37 ? 0u : (g < 95 ? 1u : 2u);
      if (gap) {
        __gmpz_set_ui(m, 1ul << (4 * gap));
        __gmpz_powm(r, o, m, c->ns);
        __gmpz_mul(t, acc, r);
      } else {
        __gmpz_mul(t, acc, o);
      }
      __gmpz_tdiv_r(acc, t, c->ns);
    }
  }
  j->secs = now_s() - t0;
  if (j->op == 5) {
    for (int k = 0; k < kSlots; ++k) __gmpz_clear(&slot[k]);
    for (int k = 0; k < kPool; ++k) __gmpz_clear(&pool[k]);
    free(slot); free(sexp); free(pool);
  }
  __gmpz_clear(m); __gmpz_clear(nude); __gmpz_clear(r); __gmpz_clear(t); __gmpz_clear(acc);
  __gmpz_clear(dp); __gmpz_clear(dq); __gmpz_clear(o);
  __gmp_randclear(rs);
  return NULL;
}

/* Run `threads` workers, each processing `per_thread` elements; returns wall seconds. */
double gref_bench(gref_ctx* c, int op, long per_thread, int threads, unsigned long seed) {
  if (threads < 1) threads = 1;
  pthread_t* th = (pthread_t*)calloc(threads, sizeof(pthread_t));
  job_t* jobs = (job_t*)calloc(threads, sizeof(job_t));
  double t0 = now_s();
  for (int i = 0; i < threads; ++i) {
    jobs[i].c = c; jobs[i].count = per_thread; jobs[i].seed = seed + 7919u * i; jobs[i].op = op;
    pthread_create(&th[i], NULL, run_job, &jobs[i]);
  }
  for (int i = 0; i < threads; ++i) pthread_join(th[i], NULL);
  double wall = now_s() - t0;
  free(th); free(jobs);
  return wall;
}
