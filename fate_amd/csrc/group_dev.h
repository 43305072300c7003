// Device grouping for the segmented ciphertext folds (fphe_fold_segments): the integer
// plumbing around the Montgomery fold kernels -- term keys, a counting sort of the terms by
// (segment, exponent), chunk tables, the per-segment exponent merge bookkeeping and the
// final scatter.  All HBM-bound byte/int work: one thread per term, key or partial, grid
// stride loops, atomics on 32-bit counters.  Included by fate_phe.hip inside its anonymous
// namespace (after set_err / kBlock).
//
// Reference: the sequential Ciphertext::add folds of iupdate / iupdate_with_masks /
// intervals_sum_with_step / matmul (fixedpoint_paillier/src/lib.rs:724-791, 861-908); the fold
// is order independent, which is what lets the terms be regrouped.

#pragma once

constexpr int kGrBlock = 256;
constexpr int32_t kI32Max = 0x7fffffff;
constexpr int32_t kI32Min = -0x7fffffff - 1;

// grid size for a one-thread-per-item integer kernel: enough blocks to fill the chip, no more
inline unsigned gr_grid(size_t n, int cus) {
  size_t g = (n + kGrBlock - 1) / kGrBlock;
  const size_t cap = (size_t)cus * 8;
  if (g > cap) g = cap;
  return (unsigned)(g ? g : 1);
}

// --- pass 1: exponent range of the terms and index bounds -------------------------------------
// mm[0] = min exponent, mm[1] = max exponent over the terms' sources (INT_MAX / INT_MIN when no
// term), mm[2] |= 1 on an index outside [0, nsrc) or a segment outside [0, nseg).
__global__ __launch_bounds__(kGrBlock) void k_gr_minmax(const int32_t* __restrict__ idx, const int32_t* __restrict__ seg,
                                                        const int32_t* __restrict__ sexp, size_t T, size_t nsrc,
                                                        size_t nseg, int32_t* __restrict__ mm) {
  int32_t lo = kI32Max, hi = kI32Min;
  int32_t bad = 0;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < T; t += (size_t)gridDim.x * blockDim.x) {
    const int32_t s = idx ? idx[t] : (int32_t)t;
    const int32_t g = seg[t];
    if (s < 0 || (size_t)s >= nsrc || g < 0 || (size_t)g >= nseg) {
      bad = 1;
      continue;
    }
    const int32_t e = sexp[s];
    lo = e < lo ? e : lo;
    hi = e > hi ? e : hi;
  }
  __shared__ int32_t slo[kGrBlock / 64], shi[kGrBlock / 64], sbad[kGrBlock / 64];
  // wave reduction, then one atomic per block
  for (int o = 32; o > 0; o >>= 1) {
    const int32_t l2 = __shfl_xor(lo, o), h2 = __shfl_xor(hi, o), b2 = __shfl_xor(bad, o);
    lo = l2 < lo ? l2 : lo;
    hi = h2 > hi ? h2 : hi;
    bad |= b2;
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    slo[w] = lo;
    shi[w] = hi;
    sbad[w] = bad;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < kGrBlock / 64; ++i) {
      lo = slo[i] < lo ? slo[i] : lo;
      hi = shi[i] > hi ? shi[i] : hi;
      bad |= sbad[i];
    }
    atomicMin(&mm[0], lo);
    atomicMax(&mm[1], hi);
    if (bad) atomicOr(&mm[2], 1);
  }
}

// --- pass 2: keys and counts ----------------------------------------------------------------
// key = seg * NE + (exp - emin).  The counters are replicated R times (cnt[key * R + c], copy
// c = (t >> 8) mod R for term t): a histogram's few hot keys take millions of atomics, and R
// copies divide that contention; the scan over the key-major copies gives every (key, copy)
// its own output range, so the scatter pass uses the same copy and needs no other change.
constexpr int kCopyShift = 8;
__global__ __launch_bounds__(kGrBlock) void k_gr_keys(const int32_t* __restrict__ idx, const int32_t* __restrict__ seg,
                                                      const int32_t* __restrict__ sexp, size_t T, int32_t emin, int32_t NE,
                                                      int32_t R, int32_t* __restrict__ keys, int32_t* __restrict__ cnt) {
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < T; t += (size_t)gridDim.x * blockDim.x) {
    const int32_t s = idx ? idx[t] : (int32_t)t;
    const int32_t k = seg[t] * NE + (sexp[s] - emin);
    keys[t] = k;
    atomicAdd(&cnt[(size_t)k * R + ((t >> kCopyShift) % R)], 1);
  }
}

// The same pass with the counts aggregated per block in LDS (key spaces up to kBcMaxKeys):
// block b owns terms [b kBcTerms, (b + 1) kBcTerms), counts them with LDS atomics and adds each
// non-zero count to cnt[key] once -- a few global atomics per key and block instead of one per
// term.  k_gr_bscatter is its scatter.
constexpr int kBcItems = 16;
constexpr int kBcTerms = kGrBlock * kBcItems;
constexpr size_t kBcMaxKeys = 16384;  // 64 KB of LDS counters
__global__ __launch_bounds__(kGrBlock) void k_gr_bkeys(const int32_t* __restrict__ idx, const int32_t* __restrict__ seg,
                                                       const int32_t* __restrict__ sexp, size_t T, int32_t emin, int32_t NE,
                                                       int32_t nkeys, int32_t* __restrict__ keys, int32_t* __restrict__ cnt) {
  extern __shared__ int32_t hist[];
  for (int32_t k = threadIdx.x; k < nkeys; k += kGrBlock) hist[k] = 0;
  __syncthreads();
  const size_t t0 = (size_t)blockIdx.x * kBcTerms + threadIdx.x;
#pragma unroll 4
  for (int i = 0; i < kBcItems; ++i) {
    const size_t t = t0 + (size_t)i * kGrBlock;
    if (t < T) {
      const int32_t src = idx ? idx[t] : (int32_t)t;
      const int32_t k = seg[t] * NE + (sexp[src] - emin);
      keys[t] = k;
      atomicAdd(&hist[k], 1);
    }
  }
  __syncthreads();
  for (int32_t k = threadIdx.x; k < nkeys; k += kGrBlock) {
    const int32_t c = hist[k];
    if (c) atomicAdd(&cnt[k], c);
  }
}

// last[seg] = the position of the segment's last term, for the segments flagged in litseg
// only (a fold that ends as the literal 1 takes its last term's exponent: the reference's
// sequential fold ends on that term, lib.rs:303-308); other segments cost one flag read
__global__ __launch_bounds__(kGrBlock) void k_gr_last(const int32_t* __restrict__ seg, size_t T,
                                                      const u8* __restrict__ litseg, int32_t* __restrict__ last) {
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < T; t += (size_t)gridDim.x * blockDim.x) {
    const int32_t g = seg[t];
    if (litseg[g]) atomicMax(&last[g], (int32_t)t);
  }
}

__global__ __launch_bounds__(kGrBlock) void k_gr_litexp(size_t nseg, const u8* __restrict__ litseg,
                                                        const int32_t* __restrict__ last, const int32_t* __restrict__ idx,
                                                        const int32_t* __restrict__ sexp, int32_t* __restrict__ eo) {
  for (size_t s = (size_t)blockIdx.x * blockDim.x + threadIdx.x; s < nseg; s += (size_t)gridDim.x * blockDim.x) {
    if (!litseg[s]) continue;
    const int32_t t = last[s];
    eo[s] = sexp[idx ? idx[t] : t];
  }
}

// nch[key] = ceil(cnt[key] / klen); stats[0] = max cnt, stats[1] = non-empty keys
__global__ __launch_bounds__(kGrBlock) void k_gr_nchunks(const int32_t* __restrict__ cnt, size_t nkeys, int32_t klen,
                                                         int32_t* __restrict__ nch, int32_t* __restrict__ stats) {
  int32_t mx = 0, nz = 0;
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < nkeys; k += (size_t)gridDim.x * blockDim.x) {
    const int32_t c = cnt[k];
    nch[k] = (c + klen - 1) / klen;
    mx = c > mx ? c : mx;
    nz += c > 0;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const int32_t m2 = __shfl_xor(mx, o);
    mx = m2 > mx ? m2 : mx;
    nz += __shfl_xor(nz, o);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMax(&stats[0], mx);
    atomicAdd(&stats[1], nz);
  }
}

// --- exclusive scan of int32 counts (3 passes; n up to 2^31 - 1 total) -------------------------
constexpr int kScanItems = 8;  // per thread
constexpr int kScanTile = kGrBlock * kScanItems;

__device__ __forceinline__ int32_t block_excl_scan(int32_t v, int32_t* total) {
  __shared__ int32_t ws[kGrBlock / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int32_t x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) ws[w] = x;
  __syncthreads();
  int32_t base = 0, tot = 0;
  for (int i = 0; i < kGrBlock / 64; ++i) {
    if (i < w) base += ws[i];
    tot += ws[i];
  }
  __syncthreads();
  *total = tot;
  return base + x - v;
}

// out[i] = exclusive prefix within the tile; bsum[tile] = tile total
__global__ __launch_bounds__(kGrBlock) void k_scan_tiles(const int32_t* __restrict__ in, size_t n,
                                                         int32_t* __restrict__ out, int32_t* __restrict__ bsum) {
  const size_t t0 = (size_t)blockIdx.x * kScanTile;
  int32_t v[kScanItems], s = 0;
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    const size_t j = t0 + (size_t)threadIdx.x * kScanItems + i;
    v[i] = j < n ? in[j] : 0;
    s += v[i];
  }
  int32_t tot;
  int32_t run = block_excl_scan(s, &tot);
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    const size_t j = t0 + (size_t)threadIdx.x * kScanItems + i;
    if (j < n) out[j] = run;
    run += v[i];
  }
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

// exclusive scan of the tile totals in one block (nb tiles, looping); total -> *total
__global__ __launch_bounds__(kGrBlock) void k_scan_sums(int32_t* __restrict__ bsum, size_t nb, int32_t* __restrict__ total) {
  int32_t carry = 0;
  for (size_t b0 = 0; b0 < nb; b0 += kGrBlock) {
    const size_t j = b0 + threadIdx.x;
    const int32_t v = j < nb ? bsum[j] : 0;
    int32_t tot;
    const int32_t ex = block_excl_scan(v, &tot);
    if (j < nb) bsum[j] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0 && total) *total = carry;
}

__global__ __launch_bounds__(kGrBlock) void k_scan_add(int32_t* __restrict__ out, size_t n, const int32_t* __restrict__ bsum) {
  const size_t t0 = (size_t)blockIdx.x * kScanTile;
  const int32_t add = bsum[blockIdx.x];
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    const size_t j = t0 + (size_t)i * kGrBlock + threadIdx.x;
    if (j < n) out[j] += add;
  }
}

// --- pass 3: counting-sort scatter ------------------------------------------------------------
// ord[off[key * R + c] + rank] = source index of the term (rank by an atomic cursor of the
// term's copy c: the order within a key is arbitrary, the fold does not depend on it)
// skey (may be null) gets the sorted keys with the term's sign in bit 31 (ssign non-null; keys
// stay below 2^25): the fold's first level then reads neither the source's sign nor its
// exponent per term (the exponent is the key's), only its row.
__global__ __launch_bounds__(kGrBlock) void k_gr_scatter(const int32_t* __restrict__ keys, const int32_t* __restrict__ idx,
                                                         const u8* __restrict__ ssign, size_t T, int32_t R,
                                                         const int32_t* __restrict__ off, int32_t* __restrict__ fill,
                                                         int32_t* __restrict__ ord, int32_t* __restrict__ skey) {
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < T; t += (size_t)gridDim.x * blockDim.x) {
    const int32_t k = keys[t];
    const size_t kc = (size_t)k * R + ((t >> kCopyShift) % R);
    const int32_t pos = off[kc] + atomicAdd(&fill[kc], 1);
    const int32_t src = idx ? idx[t] : (int32_t)t;
    ord[pos] = src;
    if (skey) skey[pos] = k | (ssign && ssign[src] ? (int32_t)0x80000000u : 0);
  }
}

// k_gr_bkeys' scatter: each term's rank within its block and key from an LDS atomic, one global
// cursor reservation per non-zero (block, key), then ord[off[key] + base + rank]
__global__ __launch_bounds__(kGrBlock) void k_gr_bscatter(const int32_t* __restrict__ keys, const int32_t* __restrict__ idx,
                                                          const u8* __restrict__ ssign, size_t T, int32_t nkeys,
                                                          const int32_t* __restrict__ off,
                                                          int32_t* __restrict__ fill, int32_t* __restrict__ ord,
                                                          int32_t* __restrict__ skey) {
  extern __shared__ int32_t hist[];
  for (int32_t k = threadIdx.x; k < nkeys; k += kGrBlock) hist[k] = 0;
  __syncthreads();
  const size_t t0 = (size_t)blockIdx.x * kBcTerms + threadIdx.x;
  int32_t kk[kBcItems], rk[kBcItems];
#pragma unroll
  for (int i = 0; i < kBcItems; ++i) {
    const size_t t = t0 + (size_t)i * kGrBlock;
    kk[i] = t < T ? keys[t] : -1;
  }
#pragma unroll
  for (int i = 0; i < kBcItems; ++i) rk[i] = kk[i] >= 0 ? atomicAdd(&hist[kk[i]], 1) : 0;
  __syncthreads();
  for (int32_t k = threadIdx.x; k < nkeys; k += kGrBlock) {
    const int32_t c = hist[k];
    if (c) hist[k] = off[k] + atomicAdd(&fill[k], c);
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kBcItems; ++i) {
    if (kk[i] < 0) continue;
    const size_t t = t0 + (size_t)i * kGrBlock;
    const int32_t pos = hist[kk[i]] + rk[i];
    const int32_t src = idx ? idx[t] : (int32_t)t;
    ord[pos] = src;
    if (skey) skey[pos] = kk[i] | (ssign && ssign[src] ? (int32_t)0x80000000u : 0);  // as k_gr_scatter
  }
}

// the same scatter for n items counted on the device, one copy, ord = item positions
__global__ __launch_bounds__(kGrBlock) void k_gr_scatter_n(const int32_t* __restrict__ keys, const int32_t* __restrict__ n_dev,
                                                           const int32_t* __restrict__ off, int32_t* __restrict__ fill,
                                                           int32_t* __restrict__ ord) {
  const size_t n = (size_t)*n_dev;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (size_t)gridDim.x * blockDim.x) {
    const int32_t k = keys[t];
    ord[off[k] + atomicAdd(&fill[k], 1)] = (int32_t)t;
  }
}

// The order in which the fold's waves take the chunks: every full chunk (klen terms) first,
// in key order, then each key's partial last chunk, longest first (a counting sort on the
// remainder) -- a wave's lanes then run chunks of about equal length.  Per key: nfull[k] =
// cnt[k] / klen, and the remainder's bucket (klen - rem) is counted in bc.
__global__ __launch_bounds__(kGrBlock) void k_gr_permcnt(const int32_t* __restrict__ cnt, size_t nkeys, int32_t klen,
                                                         int32_t* __restrict__ nfull, int32_t* __restrict__ bc) {
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < nkeys; k += (size_t)gridDim.x * blockDim.x) {
    const int32_t c = cnt[k];
    nfull[k] = c / klen;
    const int32_t r = c % klen;
    if (r) atomicAdd(&bc[klen - r], 1);
  }
}

// cperm[fulloff[k] + i] = chunk choff[k] + i (i < nfull[k]); the partial chunk of key k goes to
// NF + boff[bucket] + rank (NF = all full chunks, on the device)
__global__ __launch_bounds__(kGrBlock) void k_gr_perm(const int32_t* __restrict__ cnt, const int32_t* __restrict__ choff,
                                                      const int32_t* __restrict__ nfull,
                                                      const int32_t* __restrict__ fulloff,
                                                      const int32_t* __restrict__ nf_dev, const int32_t* __restrict__ boff,
                                                      int32_t* __restrict__ bfill, size_t nkeys, int32_t klen,
                                                      int32_t* __restrict__ cperm) {
  const int32_t NF = *nf_dev;
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < nkeys; k += (size_t)gridDim.x * blockDim.x) {
    const int32_t nfk = nfull[k], cb = choff[k], fo = fulloff[k];
    for (int32_t i = 0; i < nfk; ++i) cperm[fo + i] = cb + i;
    const int32_t r = cnt[k] % klen;
    if (r) {
      const int32_t b = klen - r;
      cperm[NF + boff[b] + atomicAdd(&bfill[b], 1)] = cb + nfk;
    }
  }
}

// The balanced first level's bookkeeping: slot i covers sorted items [i r, min((i+1) r, T)),
// or the plan's range (slot_items);
// pcnt[i] = partials it emits (1 + run changes inside its range), cnt2[key] += 1 per run
// piece (the next level's per-key item counts).
__global__ __launch_bounds__(kGrBlock) void k_gr_segcount(const int32_t* __restrict__ skey, size_t T, u32 r,
                                                          const int32_t* __restrict__ plan, int32_t* __restrict__ pcnt,
                                                          int32_t* __restrict__ cnt2) {
  const size_t nslots = plan ? (size_t)plan[1] : (T + r - 1) / r;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nslots; i += (size_t)gridDim.x * blockDim.x) {
    size_t p0, p1;
    slot_items(plan, i, T, r, p0, p1);
    if (p1 <= p0) {  // a plan's padding slot: no items, no partial
      pcnt[i] = 0;
      continue;
    }
    int32_t k = skey[p0] & 0x7fffffff, np = 1;  // bit 31: the term's sign (k_gr_bscatter)
    for (size_t p = p0 + 1; p < p1; ++p) {
      const int32_t kp = skey[p] & 0x7fffffff;
      if (kp != k) {
        atomicAdd(&cnt2[k], 1);
        k = kp;
        ++np;
      }
    }
    atomicAdd(&cnt2[k], 1);
    pcnt[i] = np;
  }
}

// keyof[pos[k]] = k for every key with flag[k] set: the non-empty keys in key order
// (k_keytree27 gives each of them its own wave)
__global__ __launch_bounds__(kGrBlock) void k_gr_keyof(const int32_t* __restrict__ flag, const int32_t* __restrict__ pos,
                                                       size_t nkeys, int32_t* __restrict__ keyof) {
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < nkeys; k += (size_t)gridDim.x * blockDim.x)
    if (flag[k]) keyof[pos[k]] = (int32_t)k;
}

// --- chunk tables: key k's items [off[k], off[k] + cnt[k]) in chunks of klen ----------------------
__global__ __launch_bounds__(kGrBlock) void k_gr_chunks(const int32_t* __restrict__ cnt, const int32_t* __restrict__ off,
                                                        const int32_t* __restrict__ choff, size_t nkeys, int32_t klen,
                                                        int32_t* __restrict__ cstart, int32_t* __restrict__ clen,
                                                        int32_t* __restrict__ ckey) {
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < nkeys; k += (size_t)gridDim.x * blockDim.x) {
    const int32_t c = cnt[k];
    const int32_t b = off[k], cb = choff[k];
    for (int32_t i = 0; i * klen < c; ++i) {
      cstart[cb + i] = b + i * klen;
      const int32_t r = c - i * klen;
      clen[cb + i] = r < klen ? r : klen;
      ckey[cb + i] = (int32_t)k;
    }
  }
}

// --- exponent merge ---------------------------------------------------------------------------------
// Per final (segment, exponent) partial p (element-major rows, L words): literal-1 test (the
// reference's zero: signed integer exactly 1, stored as M(1) = `one`) and the segment's least
// non-literal exponent.
template <int L>
// raised (may be null, per key): partials k_segfold27 already raised to an exponent chosen
// before the segment's least exponent was known -- they stay out of that minimum (k_gr_gaps
// checks the choice)
__global__ __launch_bounds__(kGrBlock) void k_gr_segmin(const u32* __restrict__ rows, const u8* __restrict__ sign,
                                                        const int32_t* __restrict__ exp, const int32_t* __restrict__ pkey,
                                                        const int32_t* __restrict__ np_dev, int32_t NE,
                                                        const u32* __restrict__ one, const u8* __restrict__ raised,
                                                        int32_t* __restrict__ segmin, u8* __restrict__ lit) {
  const int32_t np = *np_dev;
  for (size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x; p < (size_t)np; p += (size_t)gridDim.x * blockDim.x) {
    const u32* r = rows + p * L;
    u32 acc = 0;
    for (int j = 0; j < L; ++j) acc |= r[j] ^ one[j];
    const bool one = acc == 0 && sign[p] == 0;
    lit[p] = one ? 1 : 0;
    if (!one && !(raised && raised[pkey[p]])) atomicMin(&segmin[pkey[p] / NE], exp[p]);
  }
}

// gap[p] = exp - segmin (0 for literal partials and all-literal segments), exp[p] = segmin (the
// exponent every partial of the segment is aligned to), nseg-keys for the next fold, counts;
// gap beyond kMaxGap -> err (fphe_align's contract).  gmax = the largest gap (device).
// A raised partial (non-literal) must sit at or above the least exponent of the segment's
// other partials: otherwise the exponent it was raised to was below the reference's (the
// segment's least key held only literal 1s), and the call reports FPHE_EF_EXP_RANGE -- the
// caller then folds without the device merge (paillier._fold_dense), exactly.
__global__ __launch_bounds__(kGrBlock) void k_gr_gaps(int32_t* __restrict__ exp, const int32_t* __restrict__ pkey,
                                                      const u8* __restrict__ lit, const u8* __restrict__ raised,
                                                      const int32_t* __restrict__ np_dev,
                                                      int32_t NE, const int32_t* __restrict__ segmin,
                                                      int32_t* __restrict__ gap, int32_t* __restrict__ skey,
                                                      int32_t* __restrict__ scnt, int32_t* __restrict__ gmax,
                                                      int32_t* __restrict__ err) {
  const int32_t np = *np_dev;
  u32 ef = 0;
  for (size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x; p < (size_t)np; p += (size_t)gridDim.x * blockDim.x) {
    const int32_t s = pkey[p] / NE;
    const int32_t m = segmin[s];
    int32_t d = 0;
    if (raised && raised[pkey[p]] && !lit[p] && (m == kI32Max || exp[p] < m)) ef |= FPHE_EF_EXP_RANGE;
    if (m != kI32Max) {
      if (!lit[p]) {
        const long long dd = (long long)exp[p] - m;
        d = dd > kMaxGap ? kMaxGap : (int32_t)dd;
        if (dd > kMaxGap) ef |= FPHE_EF_EXP_RANGE;
      }
      exp[p] = m;
    }
    gap[p] = d;
    skey[p] = s;
    atomicAdd(&scnt[s], 1);
    if (d) atomicMax(gmax, d);
  }
  set_err(err, ef);
}

// --- raised keys and the slot plan (fphe_fold_segments; kernels27.h kRaiseMax) ---------------
// A (segment, exponent) key far above its segment's least exponent -- the reference's rare
// outliers, e.g. +-1e-30 or +-3.4e38 among gradients near 1 -- would need 4 gap squarings of its
// partial in the exponent merge, on one wave after the whole fold.  Raised keys get slots of
// their own in k_segfold27, which squares their partials there.  Candidates (one thread per
// segment): keys >= gmin exponents above the segment's least key exponent (jmin) whose
// raise_cost(gap) (4 gap squarings, in products) fits a slot (<= xmax).  Raising costs the
// whole chip about (the key's slots) x raise_cost products; leaving a key to the merge costs its
// chain, 4 gap squarings on one wave, but only the largest remaining gap counts.  So:
//   pass 1 (hist != null): per gap, the candidates' summed raise cost and their number;
//   k_gr_gapchoose: the least threshold G whose cost -- the raise costs of every candidate with
//     gap >= G plus the chain of the largest gap left -- is lowest (no raising if that wins);
//   pass 2 (gsel != null: records the keys with gap >= *gsel; null: every candidate).
// The least key may turn out to hold only literal 1s; k_gr_gaps then reports it and the
// caller folds without the device merge.
constexpr int kGapHist = 512;  // gaps with raise_cost(gap) <= xmax < kSegFoldMax: < 256
// Is source element i the literal 1 (M(1) words, sign 0)?  Tile-major words, 256 B apart.
template <int L>
__device__ __forceinline__ bool gr_is_literal(const u32* __restrict__ Src, const u8* __restrict__ ssign,
                                              const u32* __restrict__ one, int32_t i) {
  if (ssign[i]) return false;
  const u32* c = Src + ((size_t)(i >> 6) * L) * FPHE_WAVE + (i & 63);
  for (int j = 0; j < L; ++j)
    if (c[(size_t)j * FPHE_WAVE] != one[j]) return false;
  return true;
}

// The segment's least exponent among keys holding a non-literal term -- the e_min the
// reference aligns to (literal 1s are add's identity): usually the least key's first term
// settles it.  NE when the segment holds only literal 1s.
template <int L>
__device__ __forceinline__ int32_t gr_seg_jmin(const int32_t* __restrict__ c, const int32_t* __restrict__ off,
                                               size_t s, int32_t NE, const int32_t* __restrict__ ord,
                                               const u32* __restrict__ Src, const u8* __restrict__ ssign,
                                               const u32* __restrict__ one) {
  for (int32_t j = 0; j < NE; ++j) {
    if (c[j] == 0) continue;
    const int32_t o = off[s * NE + j];
    for (int32_t t = 0; t < c[j]; ++t)
      if (!gr_is_literal<L>(Src, ssign, one, ord[o + t])) return j;
  }
  return NE;
}

template <int L>
__global__ __launch_bounds__(kGrBlock) void k_gr_gapsel(const int32_t* __restrict__ cnt, const int32_t* __restrict__ off,
                                                        size_t nseg, int32_t NE, int32_t emin, int32_t gmin, int32_t xmax,
                                                        int32_t r0, const int32_t* __restrict__ ord,
                                                        const u32* __restrict__ Src, const u8* __restrict__ ssign,
                                                        const u32* __restrict__ one,
                                                        unsigned long long* __restrict__ hist,
                                                        int32_t* __restrict__ hnum, const int32_t* __restrict__ gsel,
                                                        int32_t* __restrict__ ng, int32_t* __restrict__ gkey,
                                                        int32_t* __restrict__ gcnt, int32_t* __restrict__ goff,
                                                        int32_t* __restrict__ ggap, int32_t* __restrict__ gexp) {
  const int32_t G = gsel ? *gsel : gmin;
  if (G >= NE) return;  // k_gr_gapchoose chose no raising (or no gap can reach G)
  for (size_t s = (size_t)blockIdx.x * blockDim.x + threadIdx.x; s < nseg; s += (size_t)gridDim.x * blockDim.x) {
    const int32_t* c = cnt + s * NE;
    int32_t jfirst = 0;
    while (jfirst < NE && c[jfirst] == 0) ++jfirst;
    if (jfirst + (G > gmin ? G : gmin) >= NE) continue;  // no key far enough up: nothing to check
    const int32_t jmin = gr_seg_jmin<L>(c, off, s, NE, ord, Src, ssign, one);
    for (int32_t j = jmin + (G > gmin ? G : gmin); j < NE; ++j) {
      const int32_t g = j - jmin;
      // k_segfold27 squares a raised partial at most 4 kMaxGap times: a larger gap (crafted
      // exponents only, reachable under FPHE_FOLD_RAISE=force) stays in the exponent merge,
      // whose alignment flags FPHE_EF_EXP_RANGE and refolds exactly
      if (c[j] == 0 || g > kMaxGap || raise_cost(g) > xmax) continue;
      if (hist) {
        const long long cap = r0 - raise_cost(g) > 1 ? r0 - raise_cost(g) : 1;
        const int32_t gi = g < kGapHist ? g : kGapHist - 1;
        atomicAdd(&hist[gi], (unsigned long long)(((long long)c[j] + cap - 1) / cap * raise_cost(g)));
        atomicAdd(&hnum[gi], 1);
        continue;
      }
      const int32_t h = atomicAdd(ng, 1);
      if (h >= kRaiseMax) return;
      const int32_t k = (int32_t)(s * NE) + j;
      gkey[h] = k;
      gcnt[h] = c[j];
      goff[h] = off[k];
      ggap[h] = g;
      gexp[h] = emin + jmin;
    }
  }
}

// One thread: the threshold of pass 2 (see above).  chain = the products of chip time one
// squaring on a lone wave costs (~35 us against ~1.6 ns per product chip-wide); gaps below gmin
// are never raised, so the chain left below the least threshold is bounded by gmin - 1.
__global__ void k_gr_gapchoose(const unsigned long long* __restrict__ hist, const int32_t* __restrict__ hnum,
                               int32_t gmin, long long chain, int32_t* __restrict__ gsel) {
  __shared__ int32_t below[kGapHist];  // below[G]: the largest candidate gap < G (gmin - 1: none)
  int32_t last = gmin - 1;
  for (int32_t g = 0; g < kGapHist; ++g) {
    below[g] = last;
    if (g >= gmin && hnum[g]) last = g;
  }
  int32_t gmax = 0;
  for (int32_t g = kGapHist - 1; g >= gmin; --g)
    if (hnum[g]) {
      gmax = g;
      break;
    }
  int32_t best_g = kI32Max;  // no raising
  long long best = gmax ? 4ll * gmax * chain : 0;
  long long w = 0;
  int32_t n = 0;
  for (int32_t G = gmax; G >= gmin && gmax; --G) {
    w += (long long)hist[G];
    n += hnum[G];
    if (n > kRaiseMax) break;
    const int32_t rem = below[G];  // the largest gap left to the merge
    const long long cost = w + 4ll * rem * chain;
    if (hnum[G] && cost < best) {
      best = cost;
      best_g = G;
    }
  }
  *gsel = best_g;
}

// One workgroup: the slot plan (kernels27.h) for the raised keys k_gr_gapsel found.  Regions in
// item order: stretch, raised key, stretch, ..., stretch.  A region of n items takes
// ceil(n / cap) slots, cap = r for a stretch and max(1, r - raise_cost(gap)) for a raised key,
// its items spread evenly over them (a raised slot's squarings are products in the same loop,
// so a wave mixing regions costs its longest lane, no more).  r is the least value in
// [r0, rmax] whose plan fits one round of `round` slots (rmax when none does: a multi-round
// launch).  A plan over `smax` slots falls back to the uniform one (no raised keys).
// raised[key] = 1 for the keys the plan raises.
__global__ __launch_bounds__(kGrBlock) void k_gr_plan(const int32_t* __restrict__ ng_dev, const int32_t* __restrict__ gkey,
                                                      const int32_t* __restrict__ gcnt, const int32_t* __restrict__ goff,
                                                      const int32_t* __restrict__ ggap, const int32_t* __restrict__ gexp,
                                                      int64_t T, int32_t round, int32_t r0, int32_t rmax, int32_t smax,
                                                      int32_t* __restrict__ plan, u8* __restrict__ raised) {
  __shared__ int32_t sk[kRaiseMax], sc[kRaiseMax], so[kRaiseMax], sg[kRaiseMax], se[kRaiseMax];
  __shared__ int64_t part[kGrBlock];
  __shared__ int32_t use_r;
  const int t = threadIdx.x;
  __shared__ int32_t kin[kRaiseMax];
  int32_t ng = *ng_dev;
  ng = ng < kRaiseMax ? ng : kRaiseMax;
  for (int i = t; i < ng; i += kGrBlock) kin[i] = gkey[i];
  __syncthreads();
  // rank sort by key (keys are distinct)
  for (int i = t; i < ng; i += kGrBlock) {
    const int32_t k = kin[i];
    int rk = 0;
    for (int j = 0; j < ng; ++j) rk += kin[j] < k;
    sk[rk] = k;
    sc[rk] = gcnt[i];
    so[rk] = goff[i];
    sg[rk] = ggap[i];
    se[rk] = gexp[i];
  }
  __syncthreads();
  const int nreg = 2 * ng + 1;
  auto reg = [&](int i, int64_t& st, int64_t& en, int& g) {  // region i's items and gap
    if (i & 1) {
      const int h = i >> 1;
      st = so[h];
      en = (int64_t)so[h] + sc[h];
      g = sg[h];
    } else {
      const int h = i >> 1;
      st = h == 0 ? 0 : (int64_t)so[h - 1] + sc[h - 1];
      en = h == ng ? T : (int64_t)so[h];
      g = 0;
    }
  };
  auto reg_slots = [&](int i, int64_t r, int64_t& per) -> int64_t {
    int64_t st, en;
    int g;
    reg(i, st, en, g);
    const int64_t n = en - st;
    if (n <= 0) {
      per = 1;
      return 0;
    }
    const int64_t x = g ? raise_cost(g) : 0;
    const int64_t cap = r - x > 1 ? r - x : 1;
    const int64_t ns = (n + cap - 1) / cap;
    per = (n + ns - 1) / ns;
    return ns;
  };
  auto total = [&](int64_t r) -> int64_t {  // block-wide sum of the regions' slots
    int64_t s = 0, per;
    for (int i = t; i < nreg; i += kGrBlock) s += reg_slots(i, r, per);
    part[t] = s;
    __syncthreads();
    for (int o = kGrBlock / 2; o > 0; o >>= 1) {
      if (t < o) part[t] += part[t + o];
      __syncthreads();
    }
    const int64_t v = part[0];
    __syncthreads();
    return v;
  };
  int64_t lo = r0, hi = rmax;
  if (total(rmax) > round) lo = hi = rmax;
  while (lo < hi) {  // least r with total(r) <= round (total is non-increasing in r)
    const int64_t mid = (lo + hi) / 2;
    if (total(mid) <= round) hi = mid;
    else lo = mid + 1;
  }
  const int64_t S = ng ? total(lo) : 0;
  if (t == 0) use_r = (ng == 0 || S > smax) ? -1 : (int32_t)lo;
  __syncthreads();
  int32_t* rslot = plan + 2;
  if (use_r < 0) {  // the uniform plan: one stretch at r0 items per slot
    if (t == 0) {
      plan[0] = 1;
      plan[1] = (int32_t)((T + r0 - 1) / r0);
      rslot[0] = 0;
      rslot[kPlanRegions] = 0;
      rslot[2 * kPlanRegions] = (int32_t)T;
      rslot[3 * kPlanRegions] = r0;
      rslot[4 * kPlanRegions] = 0;
      rslot[5 * kPlanRegions] = 0;
    }
    return;
  }
  for (int h = t; h < ng; h += kGrBlock) raised[sk[h]] = 1;
  // the regions' first slots: each thread a contiguous piece of the regions, then a scan of
  // the pieces' totals (64-bit divisions stay out of any serial loop)
  const int piece = (nreg + kGrBlock - 1) / kGrBlock;
  const int i0 = t * piece, i1 = i0 + piece < nreg ? i0 + piece : nreg;
  int64_t mine = 0, per;
  for (int i = i0; i < i1; ++i) mine += reg_slots(i, use_r, per);
  part[t] = mine;
  __syncthreads();
  if (t == 0) {
    int64_t acc = 0;
    for (int u = 0; u < kGrBlock; ++u) {
      const int64_t v = part[u];
      part[u] = acc;
      acc += v;
    }
    plan[0] = nreg;
    plan[1] = (int32_t)acc;
  }
  __syncthreads();
  int64_t acc = part[t];
  for (int i = i0; i < i1; ++i) {
    int64_t st, en;
    int g;
    reg(i, st, en, g);
    const int64_t ns = reg_slots(i, use_r, per);
    rslot[i] = (int32_t)acc;
    rslot[kPlanRegions + i] = (int32_t)st;
    rslot[2 * kPlanRegions + i] = (int32_t)(en > st ? en : st);
    rslot[3 * kPlanRegions + i] = (int32_t)per;
    rslot[4 * kPlanRegions + i] = g;
    rslot[5 * kPlanRegions + i] = (i & 1) ? se[i >> 1] : 0;
    acc += ns;
  }
}

// counting-sort keys for the descending-gap order of the alignment: key = gmax - gap (n on
// the device)
__global__ __launch_bounds__(kGrBlock) void k_gr_gapkeys(const int32_t* __restrict__ gap, const int32_t* __restrict__ n_dev,
                                                         int32_t gmax, int32_t* __restrict__ keys,
                                                         int32_t* __restrict__ cnt) {
  const size_t n = (size_t)*n_dev;
  for (size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (size_t)gridDim.x * blockDim.x) {
    const int32_t k = gmax - gap[p];
    keys[p] = k;
    atomicAdd(&cnt[k], 1);
  }
}

// --- element-major <-> tile-major ------------------------------------------------------------------
// One block per 64-element tile: [L][64] words (coalesced 256-B rows) -> 64 rows of L words
// (coalesced), through LDS with a 65-word row pitch.  Global loads and stores are 16 bytes a
// lane (a tile's L*64/4 of them issued before the first LDS write); the transposed LDS read
// of four limbs of one element is at most 2-way bank-conflicted at that pitch.
template <int L>
__global__ __launch_bounds__(kGrBlock) void k_tiles_to_rows(const u32* __restrict__ C, size_t count, u32* __restrict__ rows) {
  static_assert((L * FPHE_WAVE / 4) % kGrBlock == 0 && L % 4 == 0, "whole 16-byte vectors per thread");
  constexpr int kV = L * FPHE_WAVE / 4, kPer = kV / kGrBlock, kRowV = L / 4;
  __shared__ u32 t[L][FPHE_WAVE + 1];
  const size_t ntiles = (count + FPHE_WAVE - 1) / FPHE_WAVE;
  for (size_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const uint4* src = reinterpret_cast<const uint4*>(C + tile * L * FPHE_WAVE);
    uint4 v[kPer];
#pragma unroll
    for (int r = 0; r < kPer; ++r) v[r] = src[threadIdx.x + r * kGrBlock];
#pragma unroll
    for (int r = 0; r < kPer; ++r) {
      const int i = threadIdx.x + r * kGrBlock, j = i >> 4, c = (i & 15) * 4;
      t[j][c] = v[r].x;
      t[j][c + 1] = v[r].y;
      t[j][c + 2] = v[r].z;
      t[j][c + 3] = v[r].w;
    }
    __syncthreads();
    const size_t e0 = tile * FPHE_WAVE;
    const int ne = count - e0 < (size_t)FPHE_WAVE ? (int)(count - e0) : FPHE_WAVE;
    uint4* dst = reinterpret_cast<uint4*>(rows + e0 * L);
    for (int i = threadIdx.x; i < ne * kRowV; i += kGrBlock) {
      const int e = i / kRowV, k = (i % kRowV) * 4;
      dst[i] = make_uint4(t[k][e], t[k + 1][e], t[k + 2][e], t[k + 3][e]);
    }
    __syncthreads();
  }
}

// Final scatter: out[seg] (tile-major) for every segment: the segment's folded partial, or the
// literal 1 (exp 0, stored as M(1) = `one`) for a segment without terms.  A literal-1 result
// takes the exponent of the segment's last term (the reference's sequential fold ends on it,
// lib.rs:303-308).
template <int L>
__global__ __launch_bounds__(kGrBlock) void k_gr_init_out(size_t nseg, const u32* __restrict__ one, u32* __restrict__ Co,
                                                          u8* __restrict__ so, int32_t* __restrict__ eo,
                                                          u8* __restrict__ present) {
  const size_t nt = (nseg + FPHE_WAVE - 1) / FPHE_WAVE;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nt * L * FPHE_WAVE; i += (size_t)gridDim.x * blockDim.x) {
    const size_t w = (i >> 6) % L;
    Co[i] = one[w];
  }
  for (size_t s = (size_t)blockIdx.x * blockDim.x + threadIdx.x; s < nt * FPHE_WAVE; s += (size_t)gridDim.x * blockDim.x) {
    so[s] = 0;
    eo[s] = 0;
    if (present) present[s] = 0;
  }
}

template <int L>
__global__ __launch_bounds__(kGrBlock) void k_gr_final(const u32* __restrict__ rows, const u8* __restrict__ sign,
                                                       const int32_t* __restrict__ exp, const int32_t* __restrict__ pkey,
                                                       const int32_t* __restrict__ np_dev, const u32* __restrict__ one,
                                                       u8* __restrict__ litseg, u32* __restrict__ Co, u8* __restrict__ so,
                                                       int32_t* __restrict__ eo, u8* __restrict__ present) {
  const int32_t np = *np_dev;
  // one wave per partial: lanes copy words, lane 0 the per-element fields
  const size_t lane = threadIdx.x & 63;
  const size_t w0 = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, nwv = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t p = w0; p < (size_t)np; p += nwv) {
    const u32* r = rows + p * L;
    const int32_t s = pkey[p];
    u32 acc = 0;
    for (int j = (int)lane; j < L; j += 64) {
      const u32 v = r[j];
      acc |= v ^ one[j];
      Co[(((size_t)s >> 6) * L + j) * FPHE_WAVE + (s & 63)] = v;
    }
    const bool one = __ballot(acc != 0) == 0 && sign[p] == 0;
    if (lane == 0) {
      so[s] = sign[p];
      eo[s] = exp[p];  // a literal-1 result's exponent is set by k_gr_litexp
      litseg[s] = one ? 1 : 0;
      if (present) present[s] = 1;
    }
  }
}

// --- ct-add launch order (fphe_add_order) ---------------------------------------------------------
// The permutation k_add27 reads its slots through (paillier._add_order describes the why):
// the slots are cut into kAoRuns runs of whole wave tiles (one per XCD, kAddRegions), a run
// holds exactly the elements of its own element range, and inside a run
//   1. the elements whose exponent gap is >= kAoHeavy, largest gap first (a gap-31 tile is
//      ~25 ordinary tiles long: it must start early), then
//   2. block by block (kAoBlock elements), the rest by gap, largest first.
// A counting sort on (run, block, gap bin): per-block bin counts in LDS, one scan per run, an
// LDS-atomic scatter per block.  The order of equal-bin elements inside a block is whatever
// the atomics give: any order is a valid launch order (every slot computes its own element),
// so the ct-add results are the same bits.
constexpr int kAoRuns = 8;
constexpr int kAoBlock = 4096;
constexpr int kAoHeavy = 3;
constexpr int kAoBins = 64;  // bin = 63 - min(gap, 63): heavy bins [0, 61), light bins 61..63

__device__ __forceinline__ int ao_bin(const int32_t* __restrict__ ea, const int32_t* __restrict__ eb, size_t e) {
  const long long d = (long long)ea[e] - eb[e];
  const long long a = d < 0 ? -d : d;
  return 63 - (int)(a > 63 ? 63 : a);
}

// counts[(blk * kAoBins + bin)], blk = global block index (run-major: run r's blocks are
// [r * nbr, r * nbr + nbr)); one workgroup per block
__global__ __launch_bounds__(kGrBlock) void k_ao_count(const int32_t* __restrict__ ea, const int32_t* __restrict__ eb,
                                                       size_t m, size_t run, u32 nbr, int32_t* __restrict__ counts) {
  __shared__ int32_t c[kAoBins];
  const u32 blk = blockIdx.x, r = blk / nbr, b = blk % nbr;
  if (threadIdx.x < kAoBins) c[threadIdx.x] = 0;
  __syncthreads();
  const size_t e0 = (size_t)r * run + (size_t)b * kAoBlock;
  const size_t rend = (size_t)(r + 1) * run < m ? (size_t)(r + 1) * run : m;
  const size_t e1 = e0 + kAoBlock < rend ? e0 + kAoBlock : rend;
  for (size_t e = e0 + threadIdx.x; e < e1; e += kGrBlock) atomicAdd(&c[ao_bin(ea, eb, e)], 1);
  __syncthreads();
  if (threadIdx.x < kAoBins) counts[(size_t)blk * kAoBins + threadIdx.x] = c[threadIdx.x];
}

// one workgroup per run: offsets[(blk * kAoBins + bin)] = the slot of the block's first
// element of that bin.  Scan order: the heavy bins bin-major across the run's blocks, then the
// light bins block-major; each thread scans a contiguous piece of that sequence, then the
// pieces' totals are scanned in LDS.
__device__ __forceinline__ size_t ao_seq(size_t i, u32 nbr) {  // sequence position -> counter index
  const size_t nh = (size_t)(kAoBins - kAoHeavy) * nbr;
  if (i < nh) return (i % nbr) * kAoBins + i / nbr;
  const size_t j = i - nh;
  return (j / kAoHeavy) * kAoBins + (kAoBins - kAoHeavy) + j % kAoHeavy;
}

__global__ __launch_bounds__(kGrBlock) void k_ao_scan(const int32_t* __restrict__ counts, size_t run, u32 nbr,
                                                       int32_t* __restrict__ offsets) {
  __shared__ int32_t part[kGrBlock];
  const u32 r = blockIdx.x;
  const int32_t* c = counts + (size_t)r * nbr * kAoBins;
  int32_t* o = offsets + (size_t)r * nbr * kAoBins;
  const size_t total = (size_t)nbr * kAoBins, per = (total + kGrBlock - 1) / kGrBlock;
  const size_t i0 = threadIdx.x * per, i1 = i0 + per < total ? i0 + per : total;
  int32_t sum = 0;
  for (size_t i = i0; i < i1; ++i) sum += c[ao_seq(i, nbr)];
  part[threadIdx.x] = sum;
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t acc = (int32_t)((size_t)r * run);
    for (int t = 0; t < kGrBlock; ++t) {
      const int32_t v = part[t];
      part[t] = acc;
      acc += v;
    }
  }
  __syncthreads();
  int32_t pos = part[threadIdx.x];
  for (size_t i = i0; i < i1; ++i) {
    const size_t k = ao_seq(i, nbr);
    o[k] = pos;
    pos += c[k];
  }
}

__global__ __launch_bounds__(kGrBlock) void k_ao_scatter(const int32_t* __restrict__ ea, const int32_t* __restrict__ eb,
                                                         size_t m, size_t run, u32 nbr,
                                                         const int32_t* __restrict__ offsets, int32_t* __restrict__ ord) {
  __shared__ int32_t o[kAoBins];
  const u32 blk = blockIdx.x, r = blk / nbr, b = blk % nbr;
  if (threadIdx.x < kAoBins) o[threadIdx.x] = offsets[(size_t)blk * kAoBins + threadIdx.x];
  __syncthreads();
  const size_t e0 = (size_t)r * run + (size_t)b * kAoBlock;
  const size_t rend = (size_t)(r + 1) * run < m ? (size_t)(r + 1) * run : m;
  const size_t e1 = e0 + kAoBlock < rend ? e0 + kAoBlock : rend;
  for (size_t e = e0 + threadIdx.x; e < e1; e += kGrBlock) ord[atomicAdd(&o[ao_bin(ea, eb, e)], 1)] = (int32_t)e;
}
