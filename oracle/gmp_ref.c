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
 * The image ships libgmp.so.10 (6.2.1) without gmp.h, so the few entry points used are
 * declared below against GMP's documented, stable ABI (__gmpz_* symbols, mpz_t layout).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
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

/* ---------------- timed CPU baseline (same call sequence, per element) ---------------- */
typedef struct {
  gref_ctx* c;
  long count;
  unsigned long seed;
  int op;  /* 0 encrypt(obfuscated), 1 decrypt, 2 add (aligned), 3 add (Hetero-LR exponent gaps) */
  double secs;
} job_t;

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
