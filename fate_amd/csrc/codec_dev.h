// Integer and packed-float codecs (Coder, fixedpoint_paillier/src/lib.rs:68-146) on the
// device.  Included by fate_phe.hip after decode_core (one lane per element; HBM-bound).
#pragma once

namespace {

// encode_i64 / encode_i32 (lib.rs:68-78, 119-129): sig = v (v >= 0) or n + v; exp 0.
template <int L1>
__global__ __launch_bounds__(256) void k_encode_i64(KeyArgs K, const int64_t* __restrict__ x, size_t count,
                                                    u32* __restrict__ P, u8* __restrict__ neg,
                                                    int32_t* __restrict__ exp) {
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < count; e += (size_t)gridDim.x * blockDim.x) {
    const int64_t v = x[e];
    if (v >= 0) {
      P[tiled(e, L1, 0)] = (u32)(u64)v;
      P[tiled(e, L1, 1)] = (u32)((u64)v >> 32);
#pragma unroll 4
      for (int j = 2; j < L1; ++j) P[tiled(e, L1, (u32)j)] = 0u;
    } else {  // n - |v|
      const u64 mag = (u64)0 - (u64)v;
      u32 br = 0;
#pragma unroll 4
      for (int j = 0; j < L1; ++j) {
        const u32 s = j == 0 ? (u32)mag : (j == 1 ? (u32)(mag >> 32) : 0u);
        const u64 d = (u64)K.n[j] - s - br;
        P[tiled(e, L1, (u32)j)] = (u32)d;
        br = (u32)(d >> 63);
      }
    }
    neg[e] = 0;
    exp[e] = 0;
  }
}

// Signed mantissa of a decrypted significand (lib.rs:131-139): magnitude words + sign.
template <int L1>
__device__ __forceinline__ bool mantissa_core(const u32* __restrict__ P, u32 lp, size_t e, const KeyArgs& K,
                                              u32 (&M)[L1], bool& ng, u32& ef) {
  u32 br_n = 0, br_max = 0, br_nmm = 0, hi = 0;
#pragma unroll
  for (int j = 0; j < L1; ++j) {
    M[j] = (u32)j < lp ? P[tiled(e, lp, (u32)j)] : 0u;
    const u64 d0 = (u64)K.n[j] - M[j] - br_n; br_n = (u32)(d0 >> 63);
    const u64 d1 = (u64)K.max_int[j] - M[j] - br_max; br_max = (u32)(d1 >> 63);
    const u64 d2 = (u64)M[j] - K.n_mm[j] - br_nmm; br_nmm = (u32)(d2 >> 63);
  }
  for (u32 j = L1; j < lp; ++j) hi |= P[tiled(e, lp, j)];
  if (br_n || hi) { ef |= FPHE_EF_DECODE_CORRUPTED; return false; }
  ng = false;
  if (br_max == 0) return true;
  if (br_nmm == 0) {
    ng = true;
    u32 br = 0;
#pragma unroll
    for (int j = 0; j < L1; ++j) {
      const u64 d = (u64)K.n[j] - M[j] - br;
      M[j] = (u32)d; br = (u32)(d >> 63);
    }
    return true;
  }
  ef |= FPHE_EF_DECODE_OVERFLOW;
  return false;
}

// decode_i64 (lib.rs:130-142): (mantissa << 4 exp) -- a negative count is rug's floor
// shift right -- must fit i128 ("cant't convert to i128" panic), then `as i64` wraps.
template <int L1>
__global__ __launch_bounds__(256) void k_decode_i64(KeyArgs K, const u32* __restrict__ P, u32 lp,
                                                    const int32_t* __restrict__ exp, size_t count,
                                                    int64_t* __restrict__ out, int32_t* __restrict__ err) {
  u32 ef = 0;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < count; e += (size_t)gridDim.x * blockDim.x) {
    u32 M[L1];
    bool ng;
    if (!mantissa_core<L1>(P, lp, e, K, M, ng, ef)) { out[e] = 0; continue; }
    const int ex = exp[e];
    int bl = 0;  // bit length of |M|
#pragma unroll
    for (int j = 0; j < L1; ++j) if (M[j]) bl = 32 * j + 32 - __clz(M[j]);
    u64 lo = 0, hi = 0;   // |value| as 128 bits
    bool fits;
    auto word = [&](int w) -> u32 {  // word w of |M| (dynamic index, 0 outside)
      u32 r = 0;
#pragma unroll
      for (int j = 0; j < L1; ++j) r = (j == w) ? M[j] : r;
      return r;
    };
    if (ex >= 0) {
      const int s = 4 * ex;
      fits = bl == 0 || bl + s <= 128;
      if (fits && bl) {
        // |M| < 2^(128-s): assemble its low 128 bits, then shift
        const u64 m0 = ((u64)word(1) << 32) | word(0), m1 = ((u64)word(3) << 32) | word(2);
        if (s >= 128) { lo = hi = 0; }
        else if (s >= 64) { hi = m0 << (s - 64); lo = 0; }
        else if (s > 0) { hi = (m1 << s) | (m0 >> (64 - s)); lo = m0 << s; }
        else { hi = m1; lo = m0; }
      }
    } else {
      const int s = -4 * ex;
      // q = |M| >> s, rounded up for negative values (floor of the signed quotient)
      const int w0 = s >> 5, b0 = s & 31;
      auto shifted = [&](int k) -> u32 {  // word k of |M| >> s
        const u32 a = word(w0 + k), b = word(w0 + k + 1);
        return b0 ? (a >> b0) | (b << (32 - b0)) : a;
      };
      const int qbits = bl - s;
      fits = qbits <= 128;
      if (fits && qbits > 0) {
        lo = ((u64)shifted(1) << 32) | shifted(0);
        hi = ((u64)shifted(3) << 32) | shifted(2);
      }
      if (ng) {
        u32 rem = 0;
#pragma unroll
        for (int j = 0; j < L1; ++j) {
          const u32 m = (32 * j + 32 <= s) ? M[j] : ((32 * j < s) ? (M[j] & ((1u << (s - 32 * j)) - 1u)) : 0u);
          rem |= m;
        }
        if (rem) { lo += 1; if (lo == 0) hi += 1; }
      }
    }
    // i128 range: [-2^127, 2^127)
    if (fits) fits = (hi >> 63) == 0 || (ng && hi == (1ull << 63) && lo == 0);
    if (!fits) { ef |= FPHE_EF_DECODE_I128; out[e] = 0; continue; }
    out[e] = ng ? (int64_t)((u64)0 - lo) : (int64_t)lo;
  }
  set_err(err, ef);
}

// decode_i32 (lib.rs:143-146): decode_f64(...) as i32 -- Rust's saturating cast, NaN -> 0.
template <int L1>
__global__ __launch_bounds__(256) void k_decode_i32(KeyArgs K, const u32* __restrict__ P, u32 lp,
                                                    const int32_t* __restrict__ exp, size_t count,
                                                    int32_t* __restrict__ out, int32_t* __restrict__ err) {
  u32 ef = 0;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < count; e += (size_t)gridDim.x * blockDim.x) {
    const double d = decode_core<L1>(P, lp, e, exp[e], K, ef);
    int32_t v;
    if (d != d) v = 0;
    else if (d >= 2147483647.0) v = 2147483647;
    else if (d <= -2147483648.0) v = (int32_t)0x80000000;
    else v = (int32_t)d;  // truncation toward zero
    out[e] = v;
  }
  set_err(err, ef);
}

// pack_floats (lib.rs:79-93): per chunk of pack_num, acc = (acc << offset_bit) +
// round_half_away(v * 2^precision) (exact 64-bit MPFR product, ties away).  The packed
// integer is built in two's complement over L1 words; values whose scaled magnitude
// reaches 2^127 are flagged (FPHE_EF_ENCODE_NONFINITE) -- the reference's SecureBoost use
// packs g+1 and h at precision 52 (< 2^54).
template <int L1>
__global__ __launch_bounds__(64) void k_pack_f64(const double* __restrict__ x, size_t count, u32 offset_bit,
                                                 u32 pack_num, u32 precision, size_t nout, u32* __restrict__ P,
                                                 u8* __restrict__ neg, int32_t* __restrict__ exp,
                                                 int32_t* __restrict__ err) {
  u32 ef = 0;
  for (size_t c = (size_t)blockIdx.x * blockDim.x + threadIdx.x; c < nout; c += (size_t)gridDim.x * blockDim.x) {
    u32 acc[L1];
    for (int j = 0; j < L1; ++j) acc[j] = 0;
    const size_t i0 = c * pack_num;
    const u32 cnt = (u32)((count - i0) < pack_num ? (count - i0) : pack_num);
    for (u32 k = 0; k < cnt; ++k) {
      const double v = x[i0 + k];
      // r = round_half_away(v * 2^precision) as (sign, 128-bit magnitude)
      const u64 b = (u64)__double_as_longlong(v);
      const int E = (int)((b >> 52) & 0x7ff);
      const u64 frac = b & ((1ull << 52) - 1);
      const bool rneg = (b >> 63) != 0;
      if (E == 0x7ff) { ef |= FPHE_EF_ENCODE_NONFINITE; continue; }
      u64 m; int lsb;
      if (E != 0) { m = frac | (1ull << 52); lsb = E - 1075; } else { m = frac; lsb = -1074; }
      const int t = lsb + (int)precision;
      u64 rlo = 0, rhi = 0;
      if (m) {
        if (t >= 0) {
          if (t + 53 > 127) { ef |= FPHE_EF_ENCODE_NONFINITE; continue; }
          if (t >= 64) { rhi = m << (t - 64); } else if (t > 0) { rlo = m << t; rhi = m >> (64 - t); } else { rlo = m; }
        } else {
          const int s = -t;
          if (s < 64) {
            rlo = m >> s;
            const u64 rem = m & ((1ull << s) - 1), half = 1ull << (s - 1);
            if (rem >= half) rlo += 1;  // ties away from zero (magnitude)
          } else if (s == 64) {
            rlo = (m >> 63) ? 1 : 0;     // m < 2^53 < 2^63: never reaches half
          }
        }
      }
      // position of this value: offset_bit * (cnt - 1 - k)
      const u32 pos = offset_bit * (cnt - 1 - k);
      // two's complement add of (+-r) << pos into acc
      u32 rw[5] = {(u32)rlo, (u32)(rlo >> 32), (u32)rhi, (u32)(rhi >> 32), 0u};
      if (rneg) {  // negate the 160-bit value
        u32 c1 = 1;
        for (int w = 0; w < 5; ++w) { const u64 s2 = (u64)(~rw[w]) + c1; rw[w] = (u32)s2; c1 = (u32)(s2 >> 32); }
      }
      const u32 ws = pos >> 5, bs = pos & 31;
      u32 carry = 0;
      for (int j = 0; j < L1; ++j) {
        const int w = j - (int)ws;
        u32 add;
        if (w < 0) add = 0;
        else {
          const u32 a = w < 5 ? rw[w] : (rneg ? 0xffffffffu : 0u);
          const u32 bprev = w - 1 >= 0 ? (w - 1 < 5 ? rw[w - 1] : (rneg ? 0xffffffffu : 0u)) : 0u;
          add = bs ? (a << bs) | (bprev >> (32 - bs)) : a;
        }
        const u64 s2 = (u64)acc[j] + add + carry;
        acc[j] = (u32)s2;
        carry = (u32)(s2 >> 32);
      }
    }
    const bool ng = (acc[L1 - 1] >> 31) != 0;
    if (ng) {
      u32 c1 = 1;
      for (int j = 0; j < L1; ++j) { const u64 s2 = (u64)(~acc[j]) + c1; acc[j] = (u32)s2; c1 = (u32)(s2 >> 32); }
    }
    for (int j = 0; j < L1; ++j) P[tiled(c, L1, (u32)j)] = acc[j];
    neg[c] = ng ? 1 : 0;
    exp[c] = 0;
  }
  set_err(err, ef);
}

// unpack_floats (lib.rs:94-118): for packed value c, take min(remaining, pack_num) fields
// of offset_bit bits from the low end, value = trunc_to_f64(field / 2^precision)
// (Rational::to_f64, SURVEY.md §8(c) caveat: rounding toward zero), reversed per chunk.
template <int L1>
__global__ __launch_bounds__(256) void k_unpack_f64(const u32* __restrict__ P, u32 lp, size_t npacked,
                                                    u32 offset_bit, u32 pack_num, u32 precision, size_t total,
                                                    double* __restrict__ out) {
  for (size_t c = (size_t)blockIdx.x * blockDim.x + threadIdx.x; c < npacked; c += (size_t)gridDim.x * blockDim.x) {
    const size_t i0 = c * pack_num;
    if (i0 >= total) continue;
    const u32 cnt = (u32)((total - i0) < pack_num ? (total - i0) : pack_num);
    auto word = [&](u32 w) -> u32 { return w < lp ? P[tiled(c, lp, w)] : 0u; };
    for (u32 k = 0; k < cnt; ++k) {
      const u32 b0 = offset_bit * k;
      // field = bits [b0, b0 + offset_bit), at most 128 bits here
      const u32 w0 = b0 >> 5, sh = b0 & 31;
      u32 f[5];
      for (int i = 0; i < 5; ++i) {
        const u32 a = word(w0 + i), b = word(w0 + i + 1);
        f[i] = sh ? (a >> sh) | (b << (32 - sh)) : a;
      }
      const u32 nb = offset_bit < 128 ? offset_bit : 128;
      for (int i = 0; i < 4; ++i) {
        const int lowbit = 32 * i;
        if ((int)nb <= lowbit) f[i] = 0;
        else if ((int)nb < lowbit + 32) f[i] &= (1u << (nb - lowbit)) - 1u;
      }
      const u64 lo = ((u64)f[1] << 32) | f[0], hi = ((u64)f[3] << 32) | f[2];
      double v = 0.0;
      if (hi || lo) {
        const int h = hi ? 127 - __clzll(hi) : 63 - __clzll(lo);  // top bit index
        u64 mant;
        if (h > 52) {
          const int s = h - 52;  // truncate to 53 bits
          mant = s >= 64 ? (hi >> (s - 64)) : ((lo >> s) | (s ? (hi << (64 - s)) : 0));
          v = ldexp((double)mant, s - (int)precision);
        } else {
          v = ldexp((double)lo, -(int)precision);
        }
      }
      out[i0 + (cnt - 1 - k)] = v;
    }
  }
}

}  // namespace
