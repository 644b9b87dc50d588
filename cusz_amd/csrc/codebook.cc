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
// the smaller child (the right one only if strictly smaller) is strictly smaller.  Entries carry
// their frequency, so no comparison goes through the node pool (same order of operations, so
// the same heap states as the reference's pointer heap).
struct HeapEntry {
  uint64_t freq;
  int32_t id;
};

class MergeHeap {
 public:
  explicit MergeHeap(HeapEntry* q) : q_(q) {}

  void push(uint64_t f, int32_t id)
  {
    int i = end_++;
    for (int j = i >> 1; j; j = i >> 1) {
      if (q_[j].freq <= f) break;
      q_[i] = q_[j];
      i = j;
    }
    q_[i] = {f, id};
  }

  HeapEntry pop()
  {
    const HeapEntry top = q_[1];
    const HeapEntry x = q_[--end_];
    int i = 1;
    for (int l = 2; l < end_; l = 2 * i) {
      if (l + 1 < end_ && q_[l + 1].freq < q_[l].freq) l++;
      if (x.freq <= q_[l].freq) break;
      q_[i] = q_[l];
      i = l;
    }
    q_[i] = x;
    return top;
  }

  int size() const { return end_ - 1; }
  int32_t root() const { return q_[1].id; }

 private:
  HeapEntry* q_;
  int end_ = 1;
};

void limit_depth(const uint32_t* hist, int bklen, uint8_t* len)
{
  const uint64_t full = 1ull << kLmax;
  uint64_t kraft = 0;
  for (int s = 0; s < bklen; s++)
    if (len[s]) {
      len[s] = std::min<uint8_t>(len[s], kLmax);
      kraft += 1ull << (kLmax - len[s]);
    }
  while (kraft > full) {  // lengthen the deepest non-maximal, rarest (then highest) symbol
    int pick = -1;
    for (int s = 0; s < bklen; s++) {
      if (!len[s] || len[s] >= kLmax) continue;
      if (pick < 0 || len[s] > len[pick] ||
          (len[s] == len[pick] && (hist[s] < hist[pick] || (hist[s] == hist[pick] && s > pick))))
        pick = s;
    }
    kraft -= 1ull << (kLmax - len[pick] - 1);
    len[pick]++;
  }
}

}  // namespace

// code lengths; returns the longest length (0 if the histogram is empty)
int huffman_code_lengths(const uint32_t* hist, int bklen, uint8_t* len)
{
  std::memset(len, 0, bklen);
  int used = 0, only = -1;
  for (int s = 0; s < bklen; s++)
    if (hist[s]) used++, only = s;
  if (used == 0) return 0;
  if (used == 1) {
    len[only] = 1;
    return 1;
  }
  // tree nodes: leaves 0..used-1, internal nodes after them (children ids)
  thread_local std::vector<int32_t> kid;   // 2 per node
  thread_local std::vector<int32_t> sym;   // leaf symbol
  thread_local std::vector<HeapEntry> q;
  thread_local std::vector<uint8_t> depth;
  kid.resize(4 * (size_t)used), sym.resize(2 * (size_t)used), q.resize(2 * (size_t)used + 2), depth.resize(2 * (size_t)used);
  MergeHeap heap(q.data());
  int32_t nodes = 0;
  for (int s = 0; s < bklen; s++)
    if (hist[s]) {
      sym[nodes] = s, kid[2 * nodes] = -1;
      heap.push(hist[s], nodes++);
    }
  while (heap.size() > 1) {
    const HeapEntry a = heap.pop(), b = heap.pop();
    kid[2 * nodes] = a.id, kid[2 * nodes + 1] = b.id;
    heap.push(a.freq + b.freq, nodes++);
  }
  // leaf depths: parents are created after their children, so a reverse sweep from the root
  // sees every parent before its children
  int deepest = 0;
  depth[nodes - 1] = 0;
  for (int32_t id = nodes - 1; id >= 0; id--) {
    const int d = depth[id];
    if (kid[2 * id] < 0) {
      len[sym[id]] = (uint8_t)std::min(d, 255);
      deepest = std::max(deepest, d);
    }
    else {
      const int dc = std::min(d + 1, 255);
      depth[kid[2 * id]] = (uint8_t)dc, depth[kid[2 * id + 1]] = (uint8_t)dc;
    }
  }
  if (deepest > kLmax) {
    limit_depth(hist, bklen, len);
    deepest = kLmax;
  }
  return deepest;
}

// book: u32[bklen]; revbook: 4*64 + 2*bklen bytes.  Returns revbook bytes.
int build_codebook(const uint32_t* hist, int bklen, uint32_t* book, uint8_t* revbook)
{
  std::vector<uint8_t> len(bklen);
  const int max_l = huffman_code_lengths(hist, bklen, len.data());

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

  std::vector<uint16_t> keys(bklen, 0);
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
  std::memcpy(revbook + 256, keys.data(), 2 * bklen);
  return bytes;
}

}  // namespace cusz_amd
