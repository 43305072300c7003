/*
 * fate_phe.h -- C ABI of the MI355X Paillier PHE backend (libfatephe.so).
 *
 * Drop-in boundary for FATE's Paillier hot path.  Each entry point replaces one
 * vector method of the reference's pyo3 surface `fate_utils.paillier`
 * (rust/fate_utils/crates/fate_utils/src/paillier/paillier.rs) and follows the
 * arithmetic of rust/fate_utils/crates/{paillier,fixedpoint_paillier}/src/lib.rs
 * bit for bit.
 *
 * Conventions
 *  - All vector buffers are DEVICE pointers (hipMalloc'd or torch CUDA tensors),
 *    laid out limb-major ("SoA"): limb j of element e lives at buf[j * count + e].
 *    Limbs are little-endian uint32 words.
 *  - A ciphertext vector is (C, sign, exp):
 *      C    : uint32 [L2][count]   canonical residue in [0, n^2), L2 = key_bits/16
 *      sign : uint8  [count]       1 iff the reference's signed integer is C - n^2
 *      exp  : int32  [count]       base-16 fixed-point exponent
 *    The reference keeps ciphertexts as signed rug::Integer values because rug's
 *    `%` truncates; (C, sign) is that integer, losslessly.
 *  - A plaintext vector is (P, neg, exp): magnitude limbs uint32 [lp][count],
 *    neg uint8 [count] (1 = negative significand), exp int32 [count].
 *  - `stream` is a hipStream_t (NULL = default stream).  Calls are asynchronous
 *    on that stream; per-element error flags land in a device int32 word that the
 *    caller reads after synchronising.
 *  - Every function returns an fphe_status.
 */
#ifndef FATE_PHE_H
#define FATE_PHE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  FPHE_OK = 0,
  FPHE_ERR_ARG = 1,        /* bad argument (null pointer, unsupported key size, lp too large) */
  FPHE_ERR_HIP = 2,        /* HIP runtime error (allocation, launch) */
  FPHE_ERR_NO_SK = 3,      /* decrypt on a public-only context */
  FPHE_ERR_KEY = 4,        /* key material rejected (even modulus, p == q, ...) */
} fphe_status;

/* Per-element error bits written (OR-ed) into the caller's device `err` word. */
#define FPHE_EF_ENCODE_NONFINITE   0x01u  /* encode of inf/nan: reference panics in to_integer().unwrap() (fixedpoint_paillier/src/lib.rs:152-157) */
#define FPHE_EF_DECODE_CORRUPTED   0x02u  /* "Attempted to decode corrupted number" (lib.rs:171-172) */
#define FPHE_EF_DECODE_OVERFLOW    0x04u  /* "Overflow detected in decrypted number" (lib.rs:177-179) */
#define FPHE_EF_MUL_INVALID_PT     0x08u  /* "invalid plaintext" (lib.rs:342-343) */
#define FPHE_EF_NOT_INVERTIBLE     0x10u  /* invert(...).unwrap() on a non-unit (math/src/rug/mod.rs:30-35) */

typedef struct fphe_ctx fphe_ctx;

/* Create a device context for one Paillier key on HIP device `device`.
 * Replaces the key objects behind fate_utils.paillier.PK / SK
 * (paillier.rs:18-24; crates/paillier/src/lib.rs:49-69, SK::new :125-150).
 *   n      : key_bits/32 limbs (little-endian uint32), the public modulus.
 *   p, q   : key_bits/64 limbs each, or both NULL for a public-only context.
 * key_bits must be 1024 or 2048. */
fphe_status fphe_ctx_create(int device, uint32_t key_bits, const uint32_t* n,
                            const uint32_t* p, const uint32_t* q, fphe_ctx** out);
fphe_status fphe_ctx_destroy(fphe_ctx* ctx);
/* Limb counts: L2 = limbs of n^2 (ciphertext), L1 = limbs of n (plaintext). */
fphe_status fphe_ctx_limbs(const fphe_ctx* ctx, uint32_t* l2, uint32_t* l1);

/* Device-side fixed-point encode of float32 (Coder.encode_f32_vec, paillier.rs:162-169;
 * Coder::encode_f64, fixedpoint_paillier/src/lib.rs:148-168, 187-189).
 * Writes significand magnitude as 2 limbs P[2][count], neg[count], exp[count]. */
fphe_status fphe_encode_f32(const fphe_ctx* ctx, const float* x, size_t count,
                            uint32_t* P, uint8_t* neg, int32_t* exp, int32_t* err, void* stream);
/* Same for float64 (Coder.encode_f64_vec, paillier.rs:145-152). */
fphe_status fphe_encode_f64(const fphe_ctx* ctx, const double* x, size_t count,
                            uint32_t* P, uint8_t* neg, int32_t* exp, int32_t* err, void* stream);

/* Device-side decode (Coder.decode_f32_vec / decode_f64_vec, paillier.rs:153-161, 173-181;
 * Coder::decode_f64, fixedpoint_paillier/src/lib.rs:169-192).  P is [lp][count],
 * a non-negative decrypted significand (neg ignored: decrypt output is in [0,n)). */
fphe_status fphe_decode_f32(const fphe_ctx* ctx, const uint32_t* P, uint32_t lp, const int32_t* exp,
                            size_t count, float* out, int32_t* err, void* stream);
fphe_status fphe_decode_f64(const fphe_ctx* ctx, const uint32_t* P, uint32_t lp, const int32_t* exp,
                            size_t count, double* out, int32_t* err, void* stream);

/* Encrypt encoded plaintexts: PK.encrypt_encoded (paillier.rs:51-57) ->
 * fixedpoint_paillier::PK::encrypt_encoded (lib.rs:370-381) -> paillier::PK::encrypt
 * (crates/paillier/src/lib.rs:104-121).
 *   P/neg      : plaintext significands, magnitude limbs [lp][count] (lp <= L1).
 *   obfuscate  : 0 -> nude ciphertext 1+m*n (deterministic); 1 -> times r^n mod n^2.
 *   r          : NULL -> r drawn on the device from ChaCha20 keyed by rng_key[8]
 *                (uniform in [1, n-1] by rejection, as random.rs:22-25);
 *                else injected r, uint32 [L1][count] (parity/test mode).
 *   rng_nonce  : distinct per call with the same rng_key.
 * Outputs C[L2][count], sign[count].  (exp is copied by the caller.) */
fphe_status fphe_encrypt(fphe_ctx* ctx, const uint32_t* P, uint32_t lp, const uint8_t* neg,
                         size_t count, int obfuscate, const uint32_t* r,
                         const uint32_t rng_key[8], uint64_t rng_nonce,
                         uint32_t* C, uint8_t* sign, void* stream);

/* Decrypt to encoded plaintext: SK.decrypt_to_encoded (paillier.rs:79-81) ->
 * paillier::SK::decrypt (crates/paillier/src/lib.rs:163-176), CRT.
 * Output P[L1][count] in [0, n). */
fphe_status fphe_decrypt(fphe_ctx* ctx, const uint32_t* C, size_t count, uint32_t* P, void* stream);

/* Ciphertext add with exponent alignment and the literal-1 rule:
 * CiphertextVector.add (paillier.rs:343) -> Ciphertext::add (fixedpoint_paillier/src/lib.rs:301-333).
 * b_stride = 0 broadcasts element 0 of b (CiphertextVector.add_scalar, paillier.rs:346). */
fphe_status fphe_add(fphe_ctx* ctx,
                     const uint32_t* Ca, const uint8_t* sa, const int32_t* ea,
                     const uint32_t* Cb, const uint8_t* sb, const int32_t* eb, int b_stride,
                     size_t count, uint32_t* Co, uint8_t* so, int32_t* eo, void* stream);

/* Ciphertext x plaintext: CiphertextVector.mul (paillier.rs:361) -> Ciphertext::mul
 * (fixedpoint_paillier/src/lib.rs:334-349).  Plaintext (P[lp][count], neg, pexp);
 * p_stride = 0 broadcasts element 0 (mul_scalar, paillier.rs:364). */
fphe_status fphe_mul(fphe_ctx* ctx, const uint32_t* Ca, const uint8_t* sa, const int32_t* ea,
                     const uint32_t* P, uint32_t lp, const uint8_t* pneg, const int32_t* pexp, int p_stride,
                     size_t count, uint32_t* Co, uint8_t* so, int32_t* eo, int32_t* err, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* FATE_PHE_H */
