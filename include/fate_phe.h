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
 *    laid out tile-major: a vector of `count` elements of W uint32 words each is
 *    uint32 [T][W][64] with T = ceil(count/64); word j of element e lives at
 *    buf[((e/64)*W + j)*64 + e%64].  Words are little-endian (word 0 least
 *    significant).  Every 64-element tile is contiguous, so a wave reads word j of
 *    its 64 elements as one 256-byte row.  Per-element byte/int arrays (sign, neg,
 *    exp) are flat [T*64].  Buffers are padded to whole tiles.
 *  - A ciphertext vector is (C, sign, exp):
 *      C    : uint32 [T][L2][64]   the context's Montgomery-resident residue M(c) = c R mod
 *                                  n^2 (canonical, in [0, n^2)) of the canonical ciphertext
 *                                  c, R = the context's Montgomery radix (a power of two above
 *                                  n^2).  L2 = 64 for keys of at most 1024 bits, 128 up to
 *                                  2048, 256 up to 4096 (fphe_ctx_limbs)
 *      sign : uint8  [T*64]        1 iff the reference's signed integer is c - n^2
 *      exp  : int32  [T*64]        base-16 fixed-point exponent
 *    The reference keeps ciphertexts as signed rug::Integer values because rug's
 *    `%` truncates; (c, sign) is that integer, losslessly.  C is only
 *    meaningful to the context that wrote it (or one of the same key): fphe_export_signed /
 *    fphe_import_signed convert to and from the reference's integers, and the literal 1 (the
 *    reference's zero, Ciphertext::zero) is C = M(1) (fphe_ctx_mont_one).  Every product
 *    kernel works on M(.) directly, which saves the conversion product ct-add, ct x pt, the
 *    folds and the alignment each paid per element on canonical residues.
 *  - A plaintext vector is (P, neg, exp): magnitude words uint32 [T][lp][64],
 *    neg uint8 [T*64] (1 = negative significand), exp int32 [T*64].
 *  - `stream` is a hipStream_t (NULL = default stream).  Calls are asynchronous
 *    on that stream; per-element error flags land in a device int32 word that the
 *    caller reads after synchronising.  Calls with a context run on the context's device;
 *    context-less calls (fphe_permute, fphe_add_order, fphe_positions_terms, fphe_wire_*,
 *    fphe_chacha20_blocks, fphe_clock_stamp) on the device of a non-NULL `stream`, and on the
 *    calling thread's current device for NULL.
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
  FPHE_ERR_RANGE = 5,      /* fphe_fold_segments: (segment, exponent) key space too large for the
                              device grouping (nseg x exponent range > 2^25); nothing was written
                              but the initialised outputs: the caller folds another way */
} fphe_status;

/* Per-element error bits written (OR-ed) into the caller's device `err` word. */
#define FPHE_EF_ENCODE_NONFINITE   0x01u  /* encode of inf/nan: reference panics in to_integer().unwrap() (fixedpoint_paillier/src/lib.rs:152-157) */
#define FPHE_EF_DECODE_CORRUPTED   0x02u  /* "Attempted to decode corrupted number" (lib.rs:171-172) */
#define FPHE_EF_DECODE_OVERFLOW    0x04u  /* "Overflow detected in decrypted number" (lib.rs:177-179) */
#define FPHE_EF_MUL_INVALID_PT     0x08u  /* "invalid plaintext" (lib.rs:342-343) */
#define FPHE_EF_NOT_INVERTIBLE     0x10u  /* invert(...).unwrap() on a non-unit (math/src/rug/mod.rs:30-35) */
#define FPHE_EF_DECODE_I128        0x20u  /* decode_i64: "cant't convert to i128" (lib.rs:130-142) */
#define FPHE_EF_EXP_RANGE          0x40u  /* an exponent gap beyond 65536 in fphe_add or a fold (corrupt exponents) */

typedef struct fphe_ctx fphe_ctx;

/* Create a device context for one Paillier key on HIP device `device`.
 * Replaces the key objects behind fate_utils.paillier.PK / SK
 * (paillier.rs:18-24; crates/paillier/src/lib.rs:49-69, SK::new :125-150).
 *   n      : L1 limbs (little-endian uint32, zero-padded), the public modulus, bits(n) ==
 *            key_bits (paillier/src/lib.rs:82); L1 = 32 for key_bits <= 1024, 64 up to
 *            2048, else 128.
 *   p, q   : L1/2 limbs each (zero-padded), or both NULL for a public-only context.
 * key_bits: any even size 256..4096 (the reference takes any even size, lib.rs:72-87).
 * Keys below the geometry's width run its kernels with zero-padded limbs. */
fphe_status fphe_ctx_create(int device, uint32_t key_bits, const uint32_t* n,
                            const uint32_t* p, const uint32_t* q, fphe_ctx** out);
fphe_status fphe_ctx_destroy(fphe_ctx* ctx);
/* Limb counts: L2 = limbs of n^2 (ciphertext), L1 = limbs of n (plaintext). */
fphe_status fphe_ctx_limbs(const fphe_ctx* ctx, uint32_t* l2, uint32_t* l1);
/* M(1) = R mod n^2, the stored form of the literal 1 (Ciphertext::zero,
 * fixedpoint_paillier/src/lib.rs:244-249): L2 little-endian words into HOST memory. */
fphe_status fphe_ctx_mont_one(const fphe_ctx* ctx, uint32_t* one);

/* Path options of a context (not part of the reference's surface: which of two kernels with
 * the same integer results runs a call).  Small calls run one element per wave on latency
 * kernels; larger ones run the throughput kernels the bench times.
 *   FPHE_OPT_WIDE_DECRYPT_MAX    fphe_decrypt of at most this many elements: latency kernel
 *                                (default 4096, env FPHE_WIDE_DECRYPT_MAX; 0 = never)
 *   FPHE_OPT_WIDE_ENCRYPT_MAX    obfuscated fphe_encrypt likewise (default 2048)
 *   FPHE_OPT_WIDE_KH_ENCRYPT_MAX fphe_encrypt_crt with drawn (z_p, z_q) likewise (default 4096)
 *   FPHE_OPT_KH_DIRECT_Z         1: fphe_encrypt_crt with r == NULL draws (z_p, z_q); 0: draws
 *                                r and runs the two-step modexp (default 1, env
 *                                FPHE_KH_DIRECT_Z).  get returns the effective value: 0 on a
 *                                key where the direct draw is not a bijection.
 * The env variables set a new context's defaults.  Setting waits for the context's lock, so
 * it never changes a call being queued.  FPHE_ERR_ARG for an unknown option. */
enum {
  FPHE_OPT_WIDE_DECRYPT_MAX = 1,
  FPHE_OPT_WIDE_ENCRYPT_MAX = 2,
  FPHE_OPT_WIDE_KH_ENCRYPT_MAX = 3,
  FPHE_OPT_KH_DIRECT_Z = 4,
};
fphe_status fphe_ctx_set_option(fphe_ctx* ctx, int option, int64_t value);
fphe_status fphe_ctx_get_option(fphe_ctx* ctx, int option, int64_t* value);

/* Device-side fixed-point encode of float32 (Coder.encode_f32_vec, paillier.rs:162-169;
 * Coder::encode_f64, fixedpoint_paillier/src/lib.rs:148-168, 187-189).
 * Writes significand magnitude as 2 words P[T][2][64], neg, exp. */
fphe_status fphe_encode_f32(const fphe_ctx* ctx, const float* x, size_t count,
                            uint32_t* P, uint8_t* neg, int32_t* exp, int32_t* err, void* stream);
/* Same for float64 (Coder.encode_f64_vec, paillier.rs:145-152). */
fphe_status fphe_encode_f64(const fphe_ctx* ctx, const double* x, size_t count,
                            uint32_t* P, uint8_t* neg, int32_t* exp, int32_t* err, void* stream);

/* Device-side decode (Coder.decode_f32_vec / decode_f64_vec, paillier.rs:153-161, 173-181;
 * Coder::decode_f64, fixedpoint_paillier/src/lib.rs:169-192).  P is [T][lp][64],
 * a non-negative decrypted significand (neg ignored: decrypt output is in [0,n)). */
fphe_status fphe_decode_f32(const fphe_ctx* ctx, const uint32_t* P, uint32_t lp, const int32_t* exp,
                            size_t count, float* out, int32_t* err, void* stream);
fphe_status fphe_decode_f64(const fphe_ctx* ctx, const uint32_t* P, uint32_t lp, const int32_t* exp,
                            size_t count, double* out, int32_t* err, void* stream);

/* Device-side integer encode (Coder.encode_i64_vec / encode_i32_vec, paillier.rs:182-200;
 * Coder::encode_i64, fixedpoint_paillier/src/lib.rs:68-78, 119-129): sig = v (v >= 0) or
 * n + v, exp 0.  P is [T][L1][64]; i32 inputs are passed widened to int64. */
fphe_status fphe_encode_i64(const fphe_ctx* ctx, const int64_t* x, size_t count, uint32_t* P, uint8_t* neg,
                            int32_t* exp, void* stream);
/* Device-side decode to int64 (Coder.decode_i64_vec, paillier.rs:190-192; Coder::decode_i64,
 * lib.rs:130-142): (mantissa << 4 exp) with rug's floor shift for exp < 0, must fit i128
 * (else FPHE_EF_DECODE_I128), then wraps to i64. */
fphe_status fphe_decode_i64(const fphe_ctx* ctx, const uint32_t* P, uint32_t lp, const int32_t* exp, size_t count,
                            int64_t* out, int32_t* err, void* stream);
/* decode_i32 (lib.rs:143-146): decode_f64(...) as i32 (saturating, NaN -> 0). */
fphe_status fphe_decode_i32(const fphe_ctx* ctx, const uint32_t* P, uint32_t lp, const int32_t* exp, size_t count,
                            int32_t* out, int32_t* err, void* stream);
/* Coder.pack_floats (paillier.rs:135-138; lib.rs:79-93): ceil(count/pack_num) plaintexts
 * P [T][L1][64] (magnitude) + neg + exp(=0).  Scaled values must stay below 2^127. */
fphe_status fphe_pack_f64(const fphe_ctx* ctx, const double* x, size_t count, uint32_t offset_bit,
                          uint32_t pack_num, uint32_t precision, uint32_t* P, uint8_t* neg, int32_t* exp,
                          int32_t* err, void* stream);
/* Coder.unpack_floats (paillier.rs:140-142; lib.rs:94-118): `total` float64 outputs from
 * npacked plaintexts P [T][lp][64]; offset_bit <= 128. */
fphe_status fphe_unpack_f64(const fphe_ctx* ctx, const uint32_t* P, uint32_t lp, size_t npacked,
                            uint32_t offset_bit, uint32_t pack_num, uint32_t precision, size_t total,
                            double* out, void* stream);

/* Encrypt encoded plaintexts: PK.encrypt_encoded (paillier.rs:51-57) ->
 * fixedpoint_paillier::PK::encrypt_encoded (lib.rs:370-381) -> paillier::PK::encrypt
 * (crates/paillier/src/lib.rs:104-121).
 *   P/neg      : plaintext significands, magnitude words [T][lp][64] (lp <= L1).
 *   obfuscate  : 0 -> nude ciphertext 1+m*n (deterministic); 1 -> times r^n mod n^2.
 *   r          : NULL -> r drawn on the device from ChaCha20 keyed by rng_key[8]
 *                (uniform in [1, n-1] by rejection, as random.rs:22-25);
 *                else injected r, uint32 [T][L1][64] (parity/test mode).
 *   rng_nonce  : distinct per call with the same rng_key.
 * Outputs C[T][L2][64], sign.  (exp is copied by the caller.) */
fphe_status fphe_encrypt(fphe_ctx* ctx, const uint32_t* P, uint32_t lp, const uint8_t* neg,
                         size_t count, int obfuscate, const uint32_t* r,
                         const uint32_t rng_key[8], uint64_t rng_nonce,
                         uint32_t* C, uint8_t* sign, void* stream);

/* Key-holder obfuscated encryption (extension; same output as fphe_encrypt with
 * obfuscate=1 for the same r).  The reference computes r^n mod n^2 with the public key
 * alone (crates/paillier/src/lib.rs:94-98, 116); with p, q resident the same integer is
 * the CRT recombination of r^(n mod p(p-1)) mod p^2 and r^(n mod q(q-1)) mod q^2, two
 * half-width modexps (about half the multiply work).  FATE's encrypting parties
 * (Hetero-LR / SecureBoost guest, arch/context/_cipher.py) hold the private key they
 * generated.  Requires a context created with p, q (else FPHE_ERR_NO_SK); r and rng_*
 * as fphe_encrypt.  With r == NULL (device-drawn obfuscation) the library draws
 * z_p (standing for r^q mod p) and z_q (for r^p mod q) uniformly in Z_p^* x Z_q^* instead
 * of r and runs only z^s mod s^2 per half: the same distribution of r^n mod n^2 whenever
 * gcd(q, p-1) = gcd(p, q-1) = 1, checked at context creation (DESIGN.md §3;
 * FPHE_OPT_KH_DIRECT_Z = 0 draws r instead).  An injected r always gives the integers above. */
fphe_status fphe_encrypt_crt(fphe_ctx* ctx, const uint32_t* P, uint32_t lp, const uint8_t* neg,
                             size_t count, const uint32_t* r, const uint32_t rng_key[8],
                             uint64_t rng_nonce, uint32_t* C, uint8_t* sign, void* stream);

/* Decrypt to encoded plaintext: SK.decrypt_to_encoded (paillier.rs:79-81) ->
 * paillier::SK::decrypt (crates/paillier/src/lib.rs:163-176), CRT.
 * Output P[T][L1][64] in [0, n). */
fphe_status fphe_decrypt(fphe_ctx* ctx, const uint32_t* C, size_t count, uint32_t* P, void* stream);

/* Ciphertext add with exponent alignment and the literal-1 rule:
 * CiphertextVector.add (paillier.rs:343) -> Ciphertext::add (fixedpoint_paillier/src/lib.rs:301-333).
 * b_stride = 0 broadcasts element 0 of b (CiphertextVector.add_scalar, paillier.rs:346).
 * Exponent gaps |ea - eb| up to 65536 (4 x 65536 squarings of the higher-exponent operand,
 * decrese_exp_to, lib.rs:250-258) are computed exactly.  A larger gap (no encoder of the
 * reference comes near: only corrupt or crafted exponents) sets FPHE_EF_EXP_RANGE in *err
 * (err may be NULL) and leaves that element unspecified: the caller aligns such an operand
 * first with fphe_align in steps of at most 65536 (fate_amd/paillier.py does, exactly). */
fphe_status fphe_add(fphe_ctx* ctx,
                     const uint32_t* Ca, const uint8_t* sa, const int32_t* ea,
                     const uint32_t* Cb, const uint8_t* sb, const int32_t* eb, int b_stride,
                     size_t count, uint32_t* Co, uint8_t* so, int32_t* eo, int32_t* err, void* stream);

/* fphe_add computing element order[i] in launch slot i (order: DEVICE int32 [count], a
 * permutation of [0, count); NULL = identity).  Same results, element for element, as
 * fphe_add: the order only groups elements whose exponent gaps (4 squarings per step of
 * decrese_exp_to, fixedpoint_paillier/src/lib.rs:250-258) are equal, so that each wave
 * runs the squarings its own elements need.  With an order, count * L2 * 4 bytes must
 * stay below 4 GiB - 1 MiB (FPHE_ERR_ARG otherwise; fphe_add itself splits larger
 * vectors). */
fphe_status fphe_add_ordered(fphe_ctx* ctx,
                             const uint32_t* Ca, const uint8_t* sa, const int32_t* ea,
                             const uint32_t* Cb, const uint8_t* sb, const int32_t* eb, int b_stride,
                             size_t count, const int32_t* order, uint32_t* Co, uint8_t* so, int32_t* eo,
                             int32_t* err, void* stream);

/* Launch order for fphe_add_ordered over `count` element pairs (device arrays of the two
 * operands' exponents): the permutation that groups the exponent gaps |ea - eb| (every
 * element of a wave pays the wave's largest gap: 4 squarings per base-16 step, decrese_exp_to,
 * fixedpoint_paillier/src/lib.rs:250-258).  The slots are cut into 8 runs of whole wave tiles
 * (L2 = 64 / 128 / 256 sets the tile: 32 / 16 / 8 elements), one per XCD in fphe_add_ordered;
 * run r holds exactly the elements of its own element range: first those with gaps >= 3,
 * largest first, then block by block (4096 elements) the rest, largest gap first.  A device
 * counting sort, no host synchronisation.  The order within a bin is not specified (any
 * order gives the same ciphertexts).  order: int32 [count]. */
fphe_status fphe_add_order(const int32_t* ea, const int32_t* eb, size_t count, uint32_t L2, int32_t* order,
                           void* stream);

/* Ciphertext x plaintext: CiphertextVector.mul (paillier.rs:361) -> Ciphertext::mul
 * (fixedpoint_paillier/src/lib.rs:334-349).  Plaintext (P[T][lp][64], neg, pexp);
 * p_stride = 0 broadcasts element 0 (mul_scalar, paillier.rs:364). */
fphe_status fphe_mul(fphe_ctx* ctx, const uint32_t* Ca, const uint8_t* sa, const int32_t* ea,
                     const uint32_t* P, uint32_t lp, const uint8_t* pneg, const int32_t* pexp, int p_stride,
                     size_t count, uint32_t* Co, uint8_t* so, int32_t* eo, int32_t* err, void* stream);

/* Ciphertext inverse: Co = M(c^-1 mod n^2) for C = M(c) (the caller sets sign 0 and copies
 * exp).  This is the `neg` of Ciphertext::neg (fixedpoint_paillier/src/lib.rs:259-262,
 * invert via math/src/rug/mod.rs:30-35), the building block of sub / rsub
 * (CiphertextVector.sub/rsub, paillier.rs:349-358) and i_sub.  A non-unit C (the
 * reference panics in invert().unwrap()) gives Co = 0 and FPHE_EF_NOT_INVERTIBLE. */
fphe_status fphe_neg(fphe_ctx* ctx, const uint32_t* C, size_t count, uint32_t* Co, int32_t* err,
                     void* stream);

/* Segmented same-exponent fold (the ct-add fold inside CiphertextVector.iupdate /
 * iupdate_with_masks / intervals_sum_with_step / matmul, paillier.rs:300-340, 378-386;
 * fixedpoint_paillier/src/lib.rs:724-791, 861-908, Ciphertext::add :301-333): chunk i
 * folds the terms Src[ord[cstart[i] + j]], j < clen[i] (1 <= clen[i] <= 64), into
 * Co[i] = prod C mod n^2, so[i] = XOR of signs, eo[i] = the exponent of the chunk's
 * first term.  The caller groups terms by (segment, exponent): for equal exponents the
 * reference's add is exactly this product (literal 1 is its identity), and the
 * per-exponent partials are merged with fphe_add.  ord / cstart are int64 element
 * indexes, clen int32.  Src is ELEMENT-major (uint32 [count][L2], one element's words
 * contiguous: gathers then move whole 512-B elements); ssign / sexp flat; Co is the usual
 * tile-major [ceil(nchunks/64)][L2][64]. */
fphe_status fphe_fold(fphe_ctx* ctx, const uint32_t* Src, const uint8_t* ssign, const int32_t* sexp,
                      const int64_t* ord, const int64_t* cstart, const int32_t* clen, size_t nchunks,
                      uint32_t* Co, uint8_t* so, int32_t* eo, void* stream);

/* Segmented ciphertext fold with the grouping on the device: for every segment s < nseg,
 *   out[s] = Ciphertext::add-fold of Src[idx[t]] over the terms t with seg[t] == s
 * -- the sequential folds of CiphertextVector::iupdate / iupdate_with_masks (paillier.rs:
 * 261-283; fixedpoint_paillier/src/lib.rs:724-747), intervals_sum_with_step (:773-788) and the
 * matmul / rmatmul sums (:861-908), which are order independent (exponent alignment by
 * decrese_exp_to included, lib.rs:250-258,301-333).  Src is a tile-major ciphertext vector of
 * nsrc elements; idx (int32, may be NULL: term t reads element t) and seg (int32) have nterms
 * entries.  Outputs are tile-major [ceil(nseg/64)] vectors: a segment without terms gets the
 * reference's zero (the literal 1, exp 0) and present[s] = 0 (present may be NULL); a segment
 * whose fold is the literal 1 takes the exponent of its last term, as the sequential fold.
 * Every word of Co, so, eo and present (tile padding included) is written before any term is
 * read, so the caller need not initialise them.  Terms are counting-sorted by (segment, exponent) on the device, each run folded by chunked
 * Montgomery products, every segment's per-exponent partials aligned to its least exponent and
 * folded.  FPHE_ERR_ARG for an index or segment out of range; FPHE_ERR_RANGE when nseg x the
 * exponent range exceeds 2^25 buckets.  Synchronises the stream a few times (sizes). */
fphe_status fphe_fold_segments(fphe_ctx* ctx, const uint32_t* Src, const uint8_t* ssign, const int32_t* sexp,
                               size_t nsrc, const int32_t* idx, const int32_t* seg, size_t nterms, size_t nseg,
                               uint32_t* Co, uint8_t* so, int32_t* eo, uint8_t* present, int32_t* err, void* stream);

/* SecureBoost's bin indexes as fold terms: the term lists CiphertextVector::iupdate
 * (fixedpoint_paillier/src/lib.rs:724-735; paillier.rs:261-270) walks for a [ns][npos]
 * position matrix (int32, or int64 when pos_i64), sample-major: term (i, j, t), t < stride, at
 * index (i npos + j) stride + t reads src = i stride + t into slot = pos[i][j] stride + t of an
 * nslots-element histogram.  A position outside [0, nslots / stride) -- the reference's index
 * panic -- gets slot -1, which fphe_fold_segments reports as FPHE_ERR_ARG.  Writes
 * ns npos stride int32 entries to src and slot; no host sync.  FPHE_ERR_ARG when an index
 * would not fit int32. */
fphe_status fphe_positions_terms(const void* positions, int pos_i64, size_t ns, size_t npos, int32_t stride,
                                 size_t nslots, int32_t* src, int32_t* slot, void* stream);

/* Co = Ca^(2^nsq) * Cb mod n^2 with so = sb: the step of CiphertextVector::pack_squeeze
 * (paillier.rs:241-243; fixedpoint_paillier/src/lib.rs:439-450), `result.pow_mod_mut(2^shift)`
 * then `result * y % ns` (the powm result is canonical, so the product takes y's sign). */
fphe_status fphe_sqmul(fphe_ctx* ctx, const uint32_t* Ca, const uint32_t* Cb, const uint8_t* sb, uint32_t nsq,
                       size_t count, uint32_t* Co, uint8_t* so, void* stream);

/* The whole CiphertextVector::pack_squeeze (paillier.rs:241-243; fixedpoint_paillier/src/lib.rs:
 * 439-450) in one launch: for each chunk c of pack_num elements of C (the last may be short),
 * acc = x_0, then acc = acc^(2^shift_bit) * y (tdiv n^2) for each further y; Co[c] = acc and
 * so[c] = the sign the reference's integer has (x_0's for a one-element chunk, else the last
 * y's).  One chunk per wave (a latency kernel, wide_dev.h): for calls with few chunks, where
 * fphe_sqmul would run each step as a launch of nearly empty waves.  Co holds
 * ceil(count / pack_num) elements; the caller sets their exponents to 0. */
fphe_status fphe_pack_squeeze(fphe_ctx* ctx, const uint32_t* C, const uint8_t* sign, size_t count, uint32_t pack_num,
                              uint32_t shift_bit, uint32_t* Co, uint8_t* so, void* stream);

/* Co = Ca^(16^gap[i]) mod n^2 per element (gap >= 0), so = 0 where gap > 0 (canonical powm),
 * sa where gap == 0 (copied through): the exponent-alignment step of Ciphertext::add,
 * decrese_exp_to (fixedpoint_paillier/src/lib.rs:250-258), for many elements at once.  The
 * reference aligns pairwise inside its sequential folds (iupdate, intervals_sum, matmul,
 * lib.rs:521-791); aligning every per-exponent partial of a fold segment to the segment's
 * minimum exponent and multiplying gives the same integers (the fold is order-independent).
 * Elements in descending-gap order run fastest (a wave pays its largest gap).  gap is a
 * flat int32 array, each 0 <= gap <= 65536 (device memory, so the entry cannot check it: a
 * negative gap is taken as 0 and a larger one as 65536; the Python layer rejects such gaps,
 * and no exponent the reference's encoders produce comes near); C arrays tile-major as
 * fphe_add.  fphe_add likewise caps |exponent gap| at 65536. */
fphe_status fphe_align(fphe_ctx* ctx, const uint32_t* Ca, const uint8_t* sa, const int32_t* gap, size_t count,
                       uint32_t* Co, uint8_t* so, void* stream);

/* Element permutation of tile-major vectors: the data movement under CiphertextVector.slice /
 * slice_indexes / cat / i_shuffle / shuffle / iupdate and the fold plumbing (paillier.rs:
 * 228-300; fixedpoint_paillier/src/lib.rs:452-509).  scatter = 0: out[i] = in[idx[i]];
 * scatter = 1: out[idx[i]] = in[i]; for i < count.  C arrays are uint32 [ceil(n/64)][L][64];
 * sign / exp flat; any of the three components may be NULL (skipped).  Indexes outside
 * [0, nspace) are skipped.  No context: pure data movement on `stream`'s device. */
fphe_status fphe_permute(const uint32_t* Cin, const uint8_t* sin, const int32_t* ein, uint32_t L,
                         const int64_t* idx, size_t count, size_t nspace, int scatter, uint32_t* Cout,
                         uint8_t* sout, int32_t* eout, void* stream);

/* (7) The reference's signed ciphertext integers.  A reference Ciphertext holds the signed
 * rug::Integer c - sign*n^2 (truncating %, fixedpoint_paillier/src/lib.rs:24-34, 301-349;
 * paillier/src/lib.rs:35-43); this backend keeps M(c) (c canonical in [0, n^2)) and the sign.
 * export: tile-major (C, sign) -> element-major magnitude words mag[count][L2] (LSF uint32)
 * and neg[count] (1 = negative), one Montgomery product per element out of M(.); the wire /
 * pickle path and parity checks use this (CiphertextVector.__getstate__, paillier.rs:219-226).
 * import: the inverse, for |value| < n^2 (c = n^2 - |value| for a negative value), one
 * product into M(.).  Device memory beyond the caller's buffers: export works through a
 * stream-ordered scratch of at most 2^20 elements (0.5 GB at 2048 bits) whatever the count;
 * import converts in place. */
fphe_status fphe_export_signed(fphe_ctx* ctx, const uint32_t* C, const uint8_t* sign, size_t count, uint32_t* mag,
                               uint8_t* neg, void* stream);
fphe_status fphe_import_signed(fphe_ctx* ctx, const uint32_t* mag, const uint8_t* neg, size_t count, uint32_t* C,
                               uint8_t* sign, void* stream);

/* (8) Wire format of the reference's pickles: bincode 1.3 (fixint, little endian) of serde
 * structs whose big integers are rug::Integer, which rug's serde writes as {radix: i32,
 * value: String}.  Per element (fixedpoint_paillier Ciphertext / Plaintext, lib.rs:237-241,
 * 358-362): i32 radix | u64 len | "-"? digits | i32 exp; a vector is u64 count + elements
 * (CiphertextVector.__getstate__ / __setstate__, paillier.rs:219-226).  The radix follows
 * rug 1.20's serde: 10 for magnitudes of at most 32 significant bits, else 16 (lowercase).
 * The byte layout follows rug's published serde code and is not pinned against a real rug
 * build (none in this image).  No context: pure data formatting.
 *   fphe_wire_lengths: rec_len[e] = bytes of element e's record, radix[e] = 10 or 16 (device).
 *   fphe_wire_encode:  records at out + rec_off[e] (device; rec_off = exclusive scan of
 *                      the rec_len that fphe_wire_lengths wrote for the same mag / neg).
 *   fphe_wire_scan:    HOST walk of `count` records from buf + pos: digit offsets/lengths,
 *                      sign, exp, radix per element; *end = offset after the last record.
 *                      FPHE_ERR_ARG on a truncated record or a radix outside 2..36.
 *   fphe_wire_decode:  radix-16 digit strings, and radix-10 ones of at most 19 digits, ->
 *                      mag[count][L] (device); err |= 1 for a character that is not a digit
 *                      of the radix, 2 for a value wider than L words. */
fphe_status fphe_wire_lengths(const uint32_t* mag, const uint8_t* neg, uint32_t L, size_t count, int64_t* rec_len,
                              uint8_t* radix, void* stream);
fphe_status fphe_wire_encode(const uint32_t* mag, const uint8_t* neg, const int32_t* exp, uint32_t L, size_t count,
                             const int64_t* rec_off, const int64_t* rec_len, const uint8_t* radix, uint8_t* out,
                             void* stream);
fphe_status fphe_wire_scan(const uint8_t* buf, size_t nbytes, size_t pos, size_t count, int64_t* dig_off,
                           int32_t* dig_len, uint8_t* neg, int32_t* exp, int32_t* radix, size_t* end);
fphe_status fphe_wire_decode(const uint8_t* buf, const int64_t* dig_off, const int32_t* dig_len, const int32_t* radix,
                             uint32_t L, size_t count, uint32_t* mag, int32_t* err, void* stream);

/* Known-answer hook for the device CSPRNG behind the obfuscation nonces (fphe_encrypt with
 * r == NULL draws r from ChaCha20, chacha_dev.h; the reference's r comes from
 * StdRng::from_entropy(), math/src/rug/random.rs:15-25, so only the generator's correctness
 * can be pinned, not its outputs).  out[i*16 .. i*16+16) = the RFC 8439 block function of
 * (key, counter + i, nonce) for i < nblocks; out is a DEVICE buffer of 16*nblocks words.
 * The encryption kernels select element e's stream as counter = block | (e >> 32) << 16,
 * nonce = {e mod 2^32, call nonce hi, call nonce lo}. */
fphe_status fphe_chacha20_blocks(const uint32_t key[8], uint32_t counter, const uint32_t nonce[3], size_t nblocks,
                                 uint32_t* out, void* stream);

/* Diagnostics: shader-clock stamps (not part of the reference's surface; bench.py reports the
 * clock each timed leg ran at).  Queues `blocks` (1..65536) one-wave workgroups on `stream`;
 * block b writes out[3b] = the CU it ran on (XCC id << 16 | HW_ID bits 15:8: CU, SH, SE),
 * out[3b+1] = that CU's shader-clock cycle counter, out[3b+2] = the constant-rate counter,
 * whose rate in kHz goes to *wall_khz when non-NULL.  out is a DEVICE buffer of 3*blocks
 * uint64.  (c1 - c0) / (w1 - w0) * wall_khz * 1e3 over two stamps of the same CU is its mean
 * clock between them (the cycle counters of different CUs are not synchronised). */
fphe_status fphe_clock_stamp(uint64_t* out, uint32_t blocks, uint32_t* wall_khz, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* FATE_PHE_H */
