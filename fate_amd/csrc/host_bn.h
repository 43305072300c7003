// Host-side multi-precision helpers used ONLY to derive per-key Montgomery/CRT
// constants at context creation (not on any hot path).  Little-endian uint32 limbs.
#pragma once
#include <cstdint>
#include <vector>
#include <stdexcept>

namespace hbn {

using Limbs = std::vector<uint32_t>;

inline void trim(Limbs& a) { while (!a.empty() && a.back() == 0) a.pop_back(); }
inline Limbs norm(Limbs a) { trim(a); return a; }
inline bool is_zero(const Limbs& a) { for (auto w : a) if (w) return false; return true; }

inline int cmp(const Limbs& a0, const Limbs& b0) {
  Limbs a = norm(a0), b = norm(b0);
  if (a.size() != b.size()) return a.size() < b.size() ? -1 : 1;
  for (size_t i = a.size(); i-- > 0;) if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
  return 0;
}

inline Limbs add(const Limbs& a, const Limbs& b) {
  Limbs r(std::max(a.size(), b.size()) + 1, 0);
  uint64_t c = 0;
  for (size_t i = 0; i < r.size(); ++i) {
    uint64_t s = c + (i < a.size() ? a[i] : 0) + (i < b.size() ? b[i] : 0);
    r[i] = (uint32_t)s; c = s >> 32;
  }
  return norm(r);
}

// a - b, requires a >= b
inline Limbs sub(const Limbs& a, const Limbs& b) {
  Limbs r(a.size(), 0);
  int64_t br = 0;
  for (size_t i = 0; i < a.size(); ++i) {
    int64_t d = (int64_t)a[i] - (i < b.size() ? b[i] : 0) - br;
    br = d < 0; r[i] = (uint32_t)(d + (br ? ((int64_t)1 << 32) : 0));
  }
  if (br) throw std::runtime_error("hbn::sub underflow");
  return norm(r);
}

inline Limbs mul(const Limbs& a, const Limbs& b) {
  Limbs r(a.size() + b.size() + 1, 0);
  for (size_t i = 0; i < a.size(); ++i) {
    uint64_t c = 0;
    for (size_t j = 0; j < b.size(); ++j) {
      uint64_t t = (uint64_t)a[i] * b[j] + r[i + j] + c;
      r[i + j] = (uint32_t)t; c = t >> 32;
    }
    size_t k = i + b.size();
    while (c) { uint64_t t = (uint64_t)r[k] + c; r[k] = (uint32_t)t; c = t >> 32; ++k; }
  }
  return norm(r);
}

inline size_t bitlen(const Limbs& a0) {
  Limbs a = norm(a0);
  if (a.empty()) return 0;
  return (a.size() - 1) * 32 + (32 - __builtin_clz(a.back()));
}
inline bool bit(const Limbs& a, size_t i) { return i / 32 < a.size() && ((a[i / 32] >> (i % 32)) & 1); }

inline Limbs shl1(const Limbs& a) {
  Limbs r(a.size() + 1, 0);
  uint32_t c = 0;
  for (size_t i = 0; i < a.size(); ++i) { r[i] = (a[i] << 1) | c; c = a[i] >> 31; }
  r[a.size()] = c;
  return norm(r);
}

// a mod m by binary long division (setup only)
inline Limbs mod(const Limbs& a, const Limbs& m) {
  Limbs r;
  for (size_t i = bitlen(a); i-- > 0;) {
    r = shl1(r);
    if (bit(a, i)) { if (r.empty()) r.push_back(1); else r[0] |= 1; }
    if (cmp(r, m) >= 0) r = sub(r, m);
  }
  return r;
}

// 2^k mod m
inline Limbs pow2_mod(size_t k, const Limbs& m) {
  Limbs r{1};
  r = mod(r, m);
  for (size_t i = 0; i < k; ++i) { r = shl1(r); if (cmp(r, m) >= 0) r = sub(r, m); }
  return r;
}

// -m^{-1} mod 2^32 (m odd)
inline uint32_t neg_inv32(uint32_t m0) {
  uint32_t x = 1;
  for (int i = 0; i < 5; ++i) x *= 2u - m0 * x;
  return (uint32_t)(0u - x);
}

// m^{-1} mod 2^(32*k), m odd (Hensel/Newton lifting)
inline Limbs inv_pow2(const Limbs& m, size_t k) {
  // x <- x*(2 - m*x) mod 2^(32k), doubling correct bits each step
  Limbs x{0};
  uint32_t x0 = 0u - neg_inv32(m[0]);
  x[0] = x0;
  auto trunc = [&](Limbs v) { v.resize(k, 0); return norm(v); };
  for (size_t bits = 32; bits < 32 * k; bits *= 2) {
    Limbs mx = trunc(mul(trunc(m), x));
    // 2 - mx mod 2^(32k)  ==  (2^(32k) + 2 - mx) mod 2^(32k)
    Limbs two_k(k + 1, 0); two_k[k] = 1;
    Limbs t = sub(add(two_k, Limbs{2}), mx);
    x = trunc(mul(x, trunc(t)));
  }
  return trunc(x);
}

// a^{-1} mod m for odd m, gcd(a,m)=1 (binary extended Euclid); throws if not invertible
inline Limbs inv_mod(const Limbs& a0, const Limbs& m) {
  Limbs a = mod(a0, m);
  if (a.empty()) throw std::runtime_error("not invertible");
  Limbs u = a, v = m, x1{1}, x2;  // invariants: x1*a == u, x2*a == v (mod m)
  auto half_mod = [&](Limbs x) {  // x/2 mod m
    if (!x.empty() && (x[0] & 1)) x = add(x, m);
    Limbs r(x.size(), 0);
    for (size_t i = 0; i < x.size(); ++i) r[i] = (x[i] >> 1) | (i + 1 < x.size() ? x[i + 1] << 31 : 0);
    return norm(r);
  };
  auto sub_mod = [&](const Limbs& x, const Limbs& y) { return cmp(x, y) >= 0 ? sub(x, y) : sub(add(x, m), y); };
  auto one = Limbs{1};
  while (cmp(u, one) != 0 && cmp(v, one) != 0) {
    if (u.empty() || v.empty()) throw std::runtime_error("not invertible");
    while (!u.empty() && !(u[0] & 1)) {
      Limbs r(u.size(), 0);
      for (size_t i = 0; i < u.size(); ++i) r[i] = (u[i] >> 1) | (i + 1 < u.size() ? u[i + 1] << 31 : 0);
      u = norm(r); x1 = half_mod(x1);
    }
    while (!v.empty() && !(v[0] & 1)) {
      Limbs r(v.size(), 0);
      for (size_t i = 0; i < v.size(); ++i) r[i] = (v[i] >> 1) | (i + 1 < v.size() ? v[i + 1] << 31 : 0);
      v = norm(r); x2 = half_mod(x2);
    }
    if (cmp(u, v) >= 0) { u = sub(u, v); x1 = sub_mod(x1, x2); }
    else { v = sub(v, u); x2 = sub_mod(x2, x1); }
  }
  return cmp(u, one) == 0 ? mod(x1, m) : mod(x2, m);
}

inline Limbs padded(const Limbs& a, size_t n) {
  if (norm(a).size() > n) throw std::runtime_error("value does not fit");
  Limbs r = a; r.resize(n, 0); return r;
}

}  // namespace hbn
