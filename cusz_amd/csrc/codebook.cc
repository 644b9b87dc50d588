// cusz_amd/csrc/codebook.cc -- canonical Huffman codebook, built on the host.
//
// Produces exactly the reference's codebook bytes (codec/hf/src/hf_bk.seq.cc:72-145):
// code lengths come from the same binary-heap merge order (qinsert/qremove,
// hf_bk_impl1.seq.cc:103-137, leaves inserted in symbol order :192-194) -- ties between
// equal frequencies are broken by heap position, so only this exact heap reproduces the
// reference's lengths -- then canonisation as in hf_canon.seq.cc:105-161:
//   first[max] = 0, first[l] = ceil((first[l+1] + numl[l+1]) / 2),
//   the k-th used symbol (by index) of length l gets code first[l] + k,
//   book word = code | l << 27 (hf_impl.hh:40-59), unused symbols = 0xFFFFFFFF,
//   revbook = first i32[32] | entry i32[32] | keys u16[bklen].
// Two deliberate deviations (DESIGN.md "Codebook"): a lone used symbol gets a 1-bit code
// (the reference emits a 0-bit code that cannot be decoded), and trees deeper than 27 bits
// are length-limited (the reference silently emits a broken 28-bit zero code,
// hf_bk.seq.cc:108-112).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

namespace cusz_amd {

namespace {

constexpr int kLmax = 27;

// 1-based binary min-heap of tree nodes with the reference's tie-breaking (qinsert / qremove,
// hf_bk_impl1.seq.cc:103-137): a node moves up while its parent is strictly greater, down while
// the smaller child (the right one only if strictly smaller) is strictly smaller.  An entry is
// one u64, frequency << 12 | node id (frequencies are sums of u32 counts over <= 1024 symbols,
// < 2^42; ids < 2 * 1024): comparisons look at the frequency only, so the heap goes through the
// same states as the reference's pointer heap.
constexpr int kIdBits = 12;
constexpr int kMaxSym = 1 << 10;  // bklen <= 1024 (kMaxBklen)

struct MergeHeap {
  uint64_t q[2 * kMaxSym + 2];
  int end = 1;

  static uint64_t freq(uint64_t e) { return e >> kIdBits; }

  void push(uint64_t e)
  {
    const uint64_t f = freq(e);
    int i = end++;
    for (int j = i >> 1; j; j = i >> 1) {
      if (freq(q[j]) <= f) break;
      q[i] = q[j];
      i = j;
    }
    q[i] = e;
  }

  uint64_t pop()
  {
    const uint64_t top = q[1];
    const uint64_t x = q[--end], fx = freq(x);
    int i = 1;
    for (int l = 2; l < end; l = 2 * i) {
      if (l + 1 < end && freq(q[l + 1]) < freq(q[l])) l++;
      if (fx <= freq(q[l])) break;
      q[i] = q[l];
      i = l;
    }
    q[i] = x;
    return top;
  }
};

// Trees deeper than kLmax: lengthen the deepest non-maximal, rarest (then highest) symbol until
// the Kraft sum fits.  The symbol picked stays the deepest after each step, so it is lengthened
// until it reaches kLmax before another is picked, and the others keep their order: one sort
// by (length desc, count asc, symbol desc), then a walk -- the same lengths as re-scanning for
// the pick at every step (the oracle's limit_lengths, psz_oracle.c, does that).
void limit_depth(const uint32_t* hist, int bklen, uint8_t* len)
{
  const uint64_t full = 1ull << kLmax;
  uint64_t kraft = 0;
  int cand[kMaxSym], nc = 0;
  for (int s = 0; s < bklen; s++)
    if (len[s]) {
      len[s] = std::min<uint8_t>(len[s], kLmax);
      kraft += 1ull << (kLmax - len[s]);
      if (len[s] < kLmax) cand[nc++] = s;
    }
  if (kraft <= full) return;
  std::sort(cand, cand + nc, [&](int a, int b) {
    if (len[a] != len[b]) return len[a] > len[b];
    if (hist[a] != hist[b]) return hist[a] < hist[b];
    return a > b;
  });
  for (int k = 0; k < nc && kraft > full; k++) {
    const int s = cand[k];
    while (kraft > full && len[s] < kLmax) {
      kraft -= 1ull << (kLmax - len[s] - 1);
      len[s]++;
    }
  }
}

}  // namespace

// code lengths; returns the longest length (0 if the histogram is empty)
int huffman_code_lengths(const uint32_t* hist, int bklen, uint8_t* len)
{
  std::memset(len, 0, bklen);
  if (bklen > kMaxSym) return -1;
  int16_t sym[kMaxSym];  // leaf id -> symbol (leaves 0..used-1 in symbol order)
  int used = 0;
  for (int s = 0; s < bklen; s++)
    if (hist[s]) sym[used++] = (int16_t)s;
  if (used == 0) return 0;
  if (used == 1) {
    len[sym[0]] = 1;
    return 1;
  }
  MergeHeap heap;
  for (int id = 0; id < used; id++) heap.push((uint64_t)hist[sym[id]] << kIdBits | (uint64_t)id);
  // internal nodes after the leaves; parents are created after their children
  int16_t parent[2 * kMaxSym];
  int nodes = used;
  const uint64_t idmask = (1ull << kIdBits) - 1;
  while (heap.end > 2) {
    const uint64_t a = heap.pop(), b = heap.pop();
    parent[a & idmask] = (int16_t)nodes, parent[b & idmask] = (int16_t)nodes;
    heap.push((MergeHeap::freq(a) + MergeHeap::freq(b)) << kIdBits | (uint64_t)nodes);
    nodes++;
  }
  // depths by a reverse sweep from the root (every parent before its children)
  uint8_t depth[2 * kMaxSym];
  int deepest = 0;
  depth[nodes - 1] = 0;
  for (int id = nodes - 2; id >= 0; id--) {
    const int d = std::min(depth[parent[id]] + 1, 255);
    depth[id] = (uint8_t)d;
    if (id < used) {
      len[sym[id]] = (uint8_t)d;
      deepest = std::max(deepest, d);
    }
  }
  if (deepest > kLmax) {
    limit_depth(hist, bklen, len);
    deepest = kLmax;
  }
  return deepest;
}

namespace {

// canonical codes from lengths (hf_canon.seq.cc:105-161): book words code | len << 27, revbook
// = first[32] | entry[32] | symbols by (length, symbol).  Returns revbook bytes.
int canonize(const uint8_t* len, int max_l, int bklen, uint32_t* book, uint8_t* revbook)
{
  int32_t numl[32] = {0}, first[32] = {0}, entry[32] = {0}, next[32];
  for (int s = 0; s < bklen; s++)
    if (len[s]) numl[len[s]]++;
  for (int l = 1; l < 32; l++) entry[l] = entry[l - 1] + numl[l - 1];
  std::memcpy(next, entry, sizeof(next));
  if (max_l > 0) {
    first[max_l] = 0;
    for (int l = max_l - 1; l >= 1; l--) first[l] = (first[l + 1] + numl[l + 1] + 1) / 2;
  }
  first[0] = 0xff;

  uint16_t keys[kMaxSym] = {0};
  for (int s = 0; s < bklen; s++) book[s] = 0xFFFFFFFFu;
  for (int s = 0; s < bklen; s++) {
    const int l = len[s];
    if (!l) continue;
    const int slot = next[l]++;
    keys[slot] = (uint16_t)s;
    book[s] = ((uint32_t)(first[l] + slot - entry[l]) & 0x07FFFFFFu) | ((uint32_t)l << 27);
  }
  const int bytes = 4 * 64 + 2 * bklen;
  std::memset(revbook, 0, bytes);
  std::memcpy(revbook, first, 128);
  std::memcpy(revbook + 128, entry, 128);
  std::memcpy(revbook + 256, keys, 2 * bklen);
  return bytes;
}

// Two-queue Huffman code lengths (the device builder's algorithm, book_device.hh; oracle
// orc_book_twoqueue_u2): weights w = hist + smooth, used symbols stably sorted by weight (an LSD
// radix sort on (weight << 10 | symbol): no data-dependent branches), then at each merge the two
// smallest heads of the leaf queue and the internal-node queue (internal weights never
// decrease), a leaf before an internal node of equal weight.  A tree deeper than kLmax halves
// every weight ((w + 1) / 2) and is rebuilt.  Any such tree is optimal for the weights: the
// sampled codebook needs an optimal code, not the reference's heap order, and this takes a
// few microseconds where the heap's data-dependent sift branches cost 20-60 us per call on the
// benchmark host (cold branch predictor, one build per compress).
int twoqueue_lengths(const uint64_t* w, int bklen, uint8_t* len)
{
  uint64_t key[kMaxSym], tmp[kMaxSym];
  int n = 0;
  uint64_t wmax = 0;
  for (int s = 0; s < bklen; s++)
    if (w[s]) key[n++] = w[s] << 10 | (uint64_t)s, wmax = std::max(wmax, w[s]);
  std::memset(len, 0, bklen);
  if (n == 0) return 0;
  if (n == 1) {
    len[key[0] & 1023] = 1;
    return 1;
  }
  // LSD radix sort, 11-bit digits, over the bits the keys use
  int bits = 10;
  while (bits < 64 && (wmax << 10) >> bits) bits++;
  uint64_t* a = key;
  uint64_t* b = tmp;
  for (int sh = 0; sh < bits; sh += 11) {
    uint32_t cnt[2048 + 1] = {0};
    for (int i = 0; i < n; i++) cnt[((a[i] >> sh) & 2047) + 1]++;
    for (int d = 0; d < 2048; d++) cnt[d + 1] += cnt[d];
    for (int i = 0; i < n; i++) b[cnt[(a[i] >> sh) & 2047]++] = a[i];
    std::swap(a, b);
  }
  uint64_t iw[kMaxSym];
  int16_t par[2 * kMaxSym];
  int li = 0, ii = 0, ni = 0;
  while ((n - li) + (ni - ii) > 1) {
    int pick[2];
    uint64_t pw[2];
    for (int k = 0; k < 2; k++) {
      const uint64_t lw = li < n ? a[li] >> 10 : ~0ull, nw = ii < ni ? iw[ii] : ~0ull;
      const bool leaf = li < n && lw <= nw;
      pick[k] = leaf ? li : n + ii;
      pw[k] = leaf ? lw : nw;
      li += leaf, ii += !leaf;
    }
    par[pick[0]] = par[pick[1]] = (int16_t)(n + ni);
    iw[ni++] = pw[0] + pw[1];
  }
  uint8_t depth[2 * kMaxSym];
  const int root = n + ni - 1;
  int maxl = 0;
  depth[root] = 0;
  for (int id = root - 1; id >= 0; id--) {
    const int d = std::min(depth[par[id]] + 1, 255);
    depth[id] = (uint8_t)d;
    if (id < n) {
      len[a[id] & 1023] = (uint8_t)d;
      maxl = std::max(maxl, d);
    }
  }
  return maxl;
}

}  // namespace

// book: u32[bklen]; revbook: 4*64 + 2*bklen bytes.  Returns revbook bytes.
int build_codebook(const uint32_t* hist, int bklen, uint32_t* book, uint8_t* revbook)
{
  std::vector<uint8_t> len(bklen);
  const int max_l = huffman_code_lengths(hist, bklen, len.data());
  return canonize(len.data(), max_l, bklen, book, revbook);
}

// the two-queue book of hist + smooth (see twoqueue_lengths); the device builder's output
int build_codebook_twoqueue(const uint32_t* hist, int bklen, uint32_t smooth, uint32_t* book, uint8_t* revbook)
{
  if (bklen <= 0 || bklen > kMaxSym) return -1;
  uint64_t w[kMaxSym];
  uint8_t len[kMaxSym];
  for (int s = 0; s < bklen; s++) w[s] = (uint64_t)hist[s] + smooth;
  int max_l;
  while ((max_l = twoqueue_lengths(w, bklen, len)) > kLmax)
    for (int s = 0; s < bklen; s++)
      if (w[s]) w[s] = (w[s] + 1) / 2;
  return canonize(len, max_l, bklen, book, revbook);
}

}  // namespace cusz_amd
