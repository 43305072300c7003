/* Native consumer of the drop-in boundary: a plain C program (no Python, no torch) that
 * drives libfatephe.so through include/fate_phe.h the way a cgo / Rust FFI binding of
 * fate_utils.paillier would: key context, injected-r encryption of encoded
 * significands, export of the reference's signed ciphertext integers, CRT decryption.
 *
 * stdin : key_bits, n, p, q (hex), count, then `count` lines "<signed sig hex> <r hex>"
 * stdout: per element "<signed ciphertext hex> <decrypted significand hex>"
 * argv[1]: "latency" or "throughput" selects the kernels of the encrypt and the decrypt
 *          (fphe_ctx_set_option; default: the library's size thresholds)
 * tests/test_gpu_c_abi.py feeds it the golden fixture and compares with the oracle's values. */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "fate_phe.h"

#define CHECK(x)                                                       \
  do {                                                                 \
    int rc_ = (int)(x);                                                \
    if (rc_ != 0) {                                                    \
      fprintf(stderr, "%s:%d: %s -> %d\n", __FILE__, __LINE__, #x, rc_); \
      exit(2);                                                         \
    }                                                                  \
  } while (0)

/* hex string (optional leading '-') -> little-endian words; returns 1 if negative */
static int parse_hex(const char* s, uint32_t* w, size_t nw) {
  int neg = 0;
  memset(w, 0, nw * sizeof(uint32_t));
  if (*s == '-') { neg = 1; ++s; }
  if (s[0] == '0' && (s[1] == 'x' || s[1] == 'X')) s += 2;
  size_t len = strlen(s), bit = 0;
  for (size_t i = len; i-- > 0; bit += 4) {
    char c = s[i];
    uint32_t v = (c >= '0' && c <= '9') ? (uint32_t)(c - '0') : (uint32_t)((c | 32) - 'a' + 10);
    if (bit / 32 < nw) w[bit / 32] |= v << (bit % 32);
  }
  return neg;
}

static void print_hex(const uint32_t* w, size_t nw, int neg) {
  size_t top = nw;
  while (top > 1 && w[top - 1] == 0) --top;
  printf("%s0x%x", neg ? "-" : "", w[top - 1]);
  for (size_t i = top - 1; i-- > 0;) printf("%08x", w[i]);
}

static void* dalloc(size_t bytes) {
  void* p = NULL;
  CHECK(hipMalloc(&p, bytes ? bytes : 4));
  CHECK(hipMemset(p, 0, bytes ? bytes : 4));
  return p;
}

int main(int argc, char** argv) {
  unsigned bits = 0;
  size_t count = 0;
  static char buf[8192], rbuf[8192];
  if (scanf("%u", &bits) != 1) return 1;
  uint32_t n[128], p[64], q[64]; /* keys up to 4096 bits (fphe_ctx_create reads L1 <= 128 words) */
  if (scanf("%8191s", buf) != 1) return 1;
  parse_hex(buf, n, 128);
  if (scanf("%8191s", buf) != 1) return 1;
  parse_hex(buf, p, 64);
  if (scanf("%8191s", buf) != 1) return 1;
  parse_hex(buf, q, 64);
  if (scanf("%zu", &count) != 1) return 1;

  fphe_ctx* ctx = NULL;
  CHECK(fphe_ctx_create(0, bits, n, p, q, &ctx));
  if (argc > 1) {
    const int64_t wide = strcmp(argv[1], "latency") == 0 ? (int64_t)1 << 20 : 0;
    if (!wide && strcmp(argv[1], "throughput") != 0) return 1;
    CHECK(fphe_ctx_set_option(ctx, FPHE_OPT_WIDE_ENCRYPT_MAX, wide));
    CHECK(fphe_ctx_set_option(ctx, FPHE_OPT_WIDE_DECRYPT_MAX, wide));
    int64_t got = -1;
    CHECK(fphe_ctx_get_option(ctx, FPHE_OPT_WIDE_DECRYPT_MAX, &got));
    if (got != wide) return 3;
  }
  uint32_t L2 = 0, L1 = 0;
  CHECK(fphe_ctx_limbs(ctx, &L2, &L1));
  const size_t T = (count + 63) / 64;

  /* plaintext significands and nonces in the tile-major boundary layout [T][L1][64] */
  uint32_t* P = calloc(T * L1 * 64, 4);
  uint32_t* R = calloc(T * L1 * 64, 4);
  uint8_t* neg = calloc(T * 64, 1);
  uint32_t* w = calloc(L2, 4);
  for (size_t e = 0; e < count; ++e) {
    if (scanf("%8191s %8191s", buf, rbuf) != 2) return 1;
    neg[e] = (uint8_t)parse_hex(buf, w, L1);
    for (uint32_t j = 0; j < L1; ++j) P[((e / 64) * L1 + j) * 64 + e % 64] = w[j];
    parse_hex(rbuf, w, L1);
    for (uint32_t j = 0; j < L1; ++j) R[((e / 64) * L1 + j) * 64 + e % 64] = w[j];
  }
  uint32_t *dP = dalloc(T * L1 * 256), *dR = dalloc(T * L1 * 256), *dC = dalloc(T * L2 * 256);
  uint8_t *dneg = dalloc(T * 64), *dsign = dalloc(T * 64), *dmneg = dalloc(count);
  uint32_t *dmag = dalloc(count * L2 * 4), *dD = dalloc(T * L1 * 256);
  CHECK(hipMemcpy(dP, P, T * L1 * 256, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dR, R, T * L1 * 256, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dneg, neg, T * 64, hipMemcpyHostToDevice));

  CHECK(fphe_encrypt(ctx, dP, L1, dneg, count, 1, dR, NULL, 0, dC, dsign, NULL));
  CHECK(fphe_export_signed(ctx, dC, dsign, count, dmag, dmneg, NULL));
  CHECK(fphe_decrypt(ctx, dC, count, dD, NULL));
  CHECK(hipDeviceSynchronize());

  uint32_t* mag = calloc(count * L2, 4);
  uint8_t* mneg = calloc(count ? count : 1, 1);
  uint32_t* D = calloc(T * L1 * 64, 4);
  CHECK(hipMemcpy(mag, dmag, count * L2 * 4, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(mneg, dmneg, count, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(D, dD, T * L1 * 256, hipMemcpyDeviceToHost));
  for (size_t e = 0; e < count; ++e) {
    print_hex(mag + e * L2, L2, mneg[e]);
    for (uint32_t j = 0; j < L1; ++j) w[j] = D[((e / 64) * L1 + j) * 64 + e % 64];
    printf(" ");
    print_hex(w, L1, 0);
    printf("\n");
  }
  CHECK(fphe_ctx_destroy(ctx));
  hipFree(dP); hipFree(dR); hipFree(dC); hipFree(dneg); hipFree(dsign); hipFree(dmneg); hipFree(dmag); hipFree(dD);
  free(P); free(R); free(neg); free(w); free(mag); free(mneg); free(D);
  return 0;
}
