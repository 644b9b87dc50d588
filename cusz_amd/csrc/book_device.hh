// cusz_amd/csrc/book_device.hh -- canonical Huffman codebook built on the device by one
// workgroup (NT = 256 or 1024 threads; no host round trip: SURVEY.md §7.3.2).
//
// NOT the reference's heap (hf_bk_impl1.seq.cc:103-199), whose tie-breaking follows heap
// positions and only a serial heap reproduces.  Any Huffman tree has the same (minimal) total
// bit count; this one is the two-queue construction over leaves sorted by (weight, symbol), a
// leaf taken before an internal node of equal weight, computed in parallel ROUNDS:
//   s = the two smallest heads' sum; every candidate lighter than s (leaves from their sorted
//   queue, internal nodes from theirs, which never decreases) is merged in order and paired
//   consecutively -- exactly what the serial two-queue loop would pair, since every node it
//   creates meanwhile weighs at least s.  An odd candidate stays for the next round.
// (A smooth field's 1024-bin histogram needs ~24 rounds.)  Depths by pointer jumping over the
// parent links; a tree deeper than 27 bits halves every weight and is rebuilt; canonisation is
// the reference's (hf_canon.seq.cc:105-161): first[max] = 0, first[l] = ceil((first[l+1] +
// numl[l+1]) / 2), the k-th used symbol of length l (by index) gets first[l] + k, book word =
// code | l << 27, revbook = first i32[32] | entry i32[32] | keys u16[bklen].
// oracle/psz_oracle.c orc_book_twoqueue_u2 restates it serially (tests/test_gpu_book.py).
#pragma once

#include "common.hh"

namespace cusz_amd {
namespace hbook {

constexpr int kMaxSym = 1024;    // bklen <= 1024
constexpr int kThreads = 1024;   // the standalone launch's workgroup
constexpr int kLmax = 27;        // the book word's 27-bit code field (hf_impl.hh:40-59)
constexpr unsigned long long kInf = ~0ull;

struct Smem {
  unsigned long long key[kMaxSym];  // sorted leaves: weight << 11 | symbol (unused: kInf)
  unsigned long long iw[kMaxSym];   // internal node weights, creation order (non-decreasing)
  unsigned long long mw[kMaxSym];   // one round's merged candidates by rank
  uint16_t par[2 * kMaxSym];        // parent: leaves 0..n-1 (sorted order), internals n..
  uint16_t anc[2][2 * kMaxSym];     // pointer jumping
  uint16_t dep[2][2 * kMaxSym];
  uint8_t len[kMaxSym];             // code length by symbol
  uint16_t keys[kMaxSym];           // the reverse book's symbols by canonical order
  uint32_t cnt[2][2];               // a round's candidate counts (double-buffered)
  uint32_t left[2];                 // a round's odd candidate is a leaf
  uint32_t wl[kMaxSym / 64][32];    // per 64-symbol chunk and length: symbols, then their prefix
  int32_t first[32], entry[32];
  uint32_t red[16];
};

__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long v, int m)
{
  const int lo = __shfl_xor((int)(uint32_t)v, m), hi = __shfl_xor((int)(uint32_t)(v >> 32), m);
  return (unsigned long long)(uint32_t)lo | ((unsigned long long)(uint32_t)hi << 32);
}

// Bitonic sort of sm.key[0..1024) ascending.  NT = 1024: one key per thread in a register (lane
// shuffles below stride 64, LDS above); otherwise compare-exchange pairs straight in LDS.
template <int NT>
__device__ __forceinline__ void sort_keys(Smem& sm, int t)
{
  if constexpr (NT == kMaxSym) {
    unsigned long long v = sm.key[t];
    for (int k = 2; k <= kMaxSym; k <<= 1)
      for (int j = k >> 1; j > 0; j >>= 1) {
        unsigned long long o;
        if (j >= 64) {
          __syncthreads();
          sm.key[t] = v;
          __syncthreads();
          o = sm.key[t ^ j];
        }
        else
          o = shfl_xor_u64(v, j);
        const bool keep_min = ((t & j) == 0) == ((t & k) == 0);
        v = keep_min ? (o < v ? o : v) : (o > v ? o : v);
      }
    __syncthreads();
    sm.key[t] = v;
    __syncthreads();
  }
  else {
    __syncthreads();
    for (int k = 2; k <= kMaxSym; k <<= 1)
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int p = t; p < kMaxSym / 2; p += NT) {
          const int lo = (p / j) * 2 * j + (p % j), hi = lo + j;
          const unsigned long long a = sm.key[lo], b = sm.key[hi];
          const bool up = (lo & k) == 0;
          if ((a > b) == up) sm.key[lo] = b, sm.key[hi] = a;
        }
        __syncthreads();
      }
  }
}

template <int NT>
__device__ __forceinline__ uint32_t block_sum(uint32_t v, Smem& sm, int t)
{
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v += (uint32_t)__shfl_xor((int)v, d);
  __syncthreads();
  if ((t & 63) == 0) sm.red[t >> 6] = v;
  __syncthreads();
  uint32_t s = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; w++) s += sm.red[w];
  return s;
}

template <int NT>
__device__ __forceinline__ uint32_t block_max(uint32_t v, Smem& sm, int t)
{
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, d));
  __syncthreads();
  if ((t & 63) == 0) sm.red[t >> 6] = v;
  __syncthreads();
  uint32_t s = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; w++) s = max(s, sm.red[w]);
  return s;
}

// Code lengths of the n used leaves (sm.key[0..n) sorted) into sm.len[symbol]; returns the
// deepest length.  n >= 2.  Thread t holds the candidates at queue positions t + c NT.
template <int NT>
__device__ __forceinline__ uint32_t tree_lengths(Smem& sm, uint32_t n, int t)
{
  constexpr int C = kMaxSym / NT;
  auto W = [&](uint32_t i) -> unsigned long long { return sm.key[i] >> 11; };
  uint32_t li = 0, ii = 0, ni = 0;  // uniform: leaves taken, internals taken, internals made
  if (t < 2) sm.cnt[0][t] = 0, sm.cnt[1][t] = 0, sm.left[t] = 0;
  __syncthreads();
  for (uint32_t rb = 0; (n - li) + (ni - ii) > 1; rb ^= 1) {
    const unsigned long long a = li < n ? W(li) : kInf, b = li + 1 < n ? W(li + 1) : kInf;
    const unsigned long long c = ii < ni ? sm.iw[ii] : kInf, d = ii + 1 < ni ? sm.iw[ii + 1] : kInf;
    // the two smallest heads (a leaf before an internal node of equal weight)
    const unsigned long long m1 = a <= c ? a : c;
    const unsigned long long m2 = a <= c ? (b <= c ? b : c) : (a <= d ? a : d);
    const unsigned long long s = m1 + m2;
    // candidates lighter than s are prefixes of both queues; the last one of each records the count
    unsigned long long wl[C], wi[C];
    bool inL[C], inI[C];
#pragma unroll
    for (int q = 0; q < C; q++) {
      const uint32_t pl = li + (uint32_t)(t + q * NT), pi = ii + (uint32_t)(t + q * NT);
      wl[q] = pl < n ? W(pl) : kInf;
      wi[q] = pi < ni ? sm.iw[pi] : kInf;
      const unsigned long long wl1 = pl + 1 < n ? W(pl + 1) : kInf, wi1 = pi + 1 < ni ? sm.iw[pi + 1] : kInf;
      inL[q] = wl[q] < s, inI[q] = wi[q] < s;
      if (inL[q] && !(wl1 < s)) sm.cnt[rb][0] = (uint32_t)(t + q * NT) + 1;
      if (inI[q] && !(wi1 < s)) sm.cnt[rb][1] = (uint32_t)(t + q * NT) + 1;
    }
    __syncthreads();
    const uint32_t cL = sm.cnt[rb][0], cI = sm.cnt[rb][1];
    const uint32_t k = cL + cI, m = k & ~1u;  // m candidates pair up, an odd one waits
    if (t == 0) sm.cnt[rb ^ 1][0] = 0, sm.cnt[rb ^ 1][1] = 0, sm.left[rb ^ 1] = 0;
    const uint32_t parent0 = n + ni;
#pragma unroll
    for (int q = 0; q < C; q++) {
      const uint32_t pos = (uint32_t)(t + q * NT);
      if (inL[q]) {  // rank: position + internals strictly lighter (a leaf goes first on equal weight)
        uint32_t lo = 0, hi = cI;
        while (lo < hi) {
          const uint32_t mid = (lo + hi) >> 1;
          if (sm.iw[ii + mid] < wl[q]) lo = mid + 1;
          else hi = mid;
        }
        const uint32_t r = pos + lo;
        if (r < m) sm.par[li + pos] = (uint16_t)(parent0 + (r >> 1)), sm.mw[r] = wl[q];
        else sm.left[rb] = 1u;  // r == k - 1: the odd candidate is this leaf
      }
      if (inI[q]) {  // rank: position + leaves of equal or smaller weight
        uint32_t lo = 0, hi = cL;
        while (lo < hi) {
          const uint32_t mid = (lo + hi) >> 1;
          if (W(li + mid) <= wi[q]) lo = mid + 1;
          else hi = mid;
        }
        const uint32_t r = pos + lo;
        if (r < m) sm.par[n + ii + pos] = (uint16_t)(parent0 + (r >> 1)), sm.mw[r] = wi[q];
      }
    }
    __syncthreads();
    for (uint32_t q = (uint32_t)t; q < (m >> 1); q += NT) sm.iw[ni + q] = sm.mw[2 * q] + sm.mw[2 * q + 1];
    const uint32_t nl = cL - sm.left[rb];
    li += nl, ii += m - nl, ni += m >> 1;
    __syncthreads();
  }
  // depths: pointer jumping from every node to the root (the last internal node)
  const uint32_t nodes = n + ni, root = nodes - 1;
  for (uint32_t i = (uint32_t)t; i < nodes; i += NT) {
    sm.anc[0][i] = (uint16_t)(i == root ? root : sm.par[i]);
    sm.dep[0][i] = (uint16_t)(i == root ? 0u : 1u);
  }
  __syncthreads();
  int cur = 0;
  for (uint32_t span = 1; span < nodes; span <<= 1) {
    for (uint32_t i = (uint32_t)t; i < nodes; i += NT) {
      const uint32_t a = sm.anc[cur][i];
      sm.dep[cur ^ 1][i] = (uint16_t)(sm.dep[cur][i] + sm.dep[cur][a]);
      sm.anc[cur ^ 1][i] = sm.anc[cur][a];
    }
    cur ^= 1;
    __syncthreads();
  }
  uint32_t deepest = 0;
  for (uint32_t i = (uint32_t)t; i < n; i += NT) {
    const uint32_t d = sm.dep[cur][i];
    sm.len[sm.key[i] & 2047u] = (uint8_t)min(d, 255u);
    deepest = max(deepest, d);
  }
  return block_max<NT>(deepest, sm, t);
}

// Book and reverse book of the histogram (+ smooth per bin) into global memory.  Every thread of
// the NT-thread workgroup calls it; `hist` may be global or LDS.
template <int NT>
__device__ __forceinline__ void build(const uint32_t* hist, int bklen, uint32_t smooth, uint32_t* book, uint8_t* revbook,
                                      Smem& sm)
{
  static_assert(NT == 256 || NT == 1024, "workgroup size");
  constexpr int C = kMaxSym / NT;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  unsigned long long w[C];
#pragma unroll
  for (int q = 0; q < C; q++) {
    const int s = t + q * NT;
    w[q] = s < bklen ? (unsigned long long)hist[s] + smooth : 0ull;
  }
  uint32_t maxl = 0;
  for (;;) {  // (repeats only when a tree is deeper than kLmax: weights halved)
    uint32_t used = 0;
#pragma unroll
    for (int q = 0; q < C; q++) {
      const int s = t + q * NT;
      sm.len[s] = 0;
      sm.key[s] = w[q] ? (w[q] << 11 | (unsigned long long)s) : kInf;
      used += w[q] ? 1u : 0u;
    }
    const uint32_t n = block_sum<NT>(used, sm, t);
    sort_keys<NT>(sm, t);
    if (n == 0) break;
    if (n == 1) {
      if (t == 0) sm.len[sm.key[0] & 2047u] = 1;
      maxl = 1;
      break;
    }
    maxl = tree_lengths<NT>(sm, n, t);
    if (maxl <= (uint32_t)kLmax) break;
#pragma unroll
    for (int q = 0; q < C; q++) w[q] = w[q] ? (w[q] + 1) >> 1 : 0ull;
    __syncthreads();
  }
  __syncthreads();
  // canonisation: rank of each symbol among the same length's symbols, by symbol index
  // (symbol t + q NT lies in 64-symbol chunk q (NT / 64) + wid)
  uint32_t l[C], rank[C];
  const uint64_t lt = (1ull << lane) - 1ull;
#pragma unroll
  for (int q = 0; q < C; q++) {
    l[q] = sm.len[t + q * NT];
    rank[q] = 0;
    const int ch = q * (NT / 64) + wid;
    for (uint32_t b = 1; b <= maxl; b++) {
      const uint64_t msk = __ballot(l[q] == b);
      if (l[q] == b) rank[q] = (uint32_t)__popcll(msk & lt);
      if (lane == 0) sm.wl[ch][b] = (uint32_t)__popcll(msk);
    }
  }
  __syncthreads();
  if (t < 32) {  // per length: exclusive prefix over the chunks (in place) and the total
    uint32_t acc = 0;
    for (int v = 0; v < kMaxSym / 64; v++) {
      const uint32_t c = (uint32_t)t <= maxl && t > 0 ? sm.wl[v][t] : 0u;
      sm.wl[v][t] = acc;
      acc += c;
    }
    sm.entry[t] = (int32_t)acc;  // numl[t] for now
  }
  __syncthreads();
  if (t == 0) {
    int32_t numl[32], e = 0;
    for (int q = 0; q < 32; q++) numl[q] = sm.entry[q];
    for (int q = 0; q < 32; q++) {  // entry[q] = symbols shorter than q
      sm.entry[q] = e;
      e += numl[q];
    }
    for (int q = 0; q < 32; q++) sm.first[q] = 0;
    if (maxl > 0) {
      sm.first[maxl] = 0;
      for (int q = (int)maxl - 1; q >= 1; q--) sm.first[q] = (sm.first[q + 1] + numl[q + 1] + 1) / 2;
    }
    sm.first[0] = 0xff;
  }
#pragma unroll
  for (int q = 0; q < C; q++) sm.keys[t + q * NT] = 0;  // unused tail
  __syncthreads();
#pragma unroll
  for (int q = 0; q < C; q++) {
    const int s = t + q * NT;
    if (s >= bklen) continue;
    if (l[q]) {
      const uint32_t k = sm.wl[q * (NT / 64) + wid][l[q]] + rank[q];
      book[s] = ((uint32_t)(sm.first[l[q]] + (int32_t)k) & 0x07FFFFFFu) | (l[q] << 27);
      sm.keys[sm.entry[l[q]] + (int32_t)k] = (uint16_t)s;
    }
    else
      book[s] = 0xFFFFFFFFu;
  }
  if (t < 32) {
    reinterpret_cast<int32_t*>(revbook)[t] = sm.first[t];
    reinterpret_cast<int32_t*>(revbook + 128)[t] = sm.entry[t];
  }
  __syncthreads();
  for (int s = t; s < bklen; s += NT) reinterpret_cast<uint16_t*>(revbook + 256)[s] = sm.keys[s];
}

}  // namespace hbook
}  // namespace cusz_amd
