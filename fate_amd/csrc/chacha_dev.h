// Device ChaCha20 block function (RFC 8439) used as the CSPRNG for the obfuscation
// nonce r of Paillier encryption.  The reference draws r from a fresh
// StdRng::from_entropy() per element (rust/fate_utils/crates/math/src/rug/random.rs:15-25);
// here each element owns an independent ChaCha20 stream selected by
// (context key, call nonce, element index, attempt) -- no two elements share a block.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fphe {

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

#define FPHE_QR(a, b, c, d)                    \
  a += b; d ^= a; d = rotl32(d, 16);           \
  c += d; b ^= c; b = rotl32(b, 12);           \
  a += b; d ^= a; d = rotl32(d, 8);            \
  c += d; b ^= c; b = rotl32(b, 7);

struct ChaChaKey { uint32_t k[8]; };

__device__ __forceinline__ void chacha20_block(const ChaChaKey& key, uint32_t counter, uint32_t n0,
                                               uint32_t n1, uint32_t n2, uint32_t (&out)[16]) {
  uint32_t x[16];
  x[0] = 0x61707865u; x[1] = 0x3320646eu; x[2] = 0x79622d32u; x[3] = 0x6b206574u;
#pragma unroll
  for (int i = 0; i < 8; ++i) x[4 + i] = key.k[i];
  x[12] = counter; x[13] = n0; x[14] = n1; x[15] = n2;
  uint32_t s[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) s[i] = x[i];
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    FPHE_QR(x[0], x[4], x[8], x[12]);
    FPHE_QR(x[1], x[5], x[9], x[13]);
    FPHE_QR(x[2], x[6], x[10], x[14]);
    FPHE_QR(x[3], x[7], x[11], x[15]);
    FPHE_QR(x[0], x[5], x[10], x[15]);
    FPHE_QR(x[1], x[6], x[11], x[12]);
    FPHE_QR(x[2], x[7], x[8], x[13]);
    FPHE_QR(x[3], x[4], x[9], x[14]);
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) out[i] = x[i] + s[i];
}

#undef FPHE_QR

}  // namespace fphe
