// cusz_amd/csrc/kernels.hh -- launchers of the hand-written gfx950 kernels.
#pragma once

#include "common.hh"

namespace cusz_amd {

struct XferRegions {
  int count;
  int nwords[4];
  uint32_t* dst[4];
  const uint32_t* src[4];
};
// Words the last workgroup of a kernel copies to the host before raising a host flag (the
// kernel's own publish: no separate launch; pub_device.hh publish_last).  ticket: 9 words zeroed
// before the launch.
struct HostPub {
  XferRegions r{};
  uint32_t* flag = nullptr;  // null: no publish
  uint32_t epoch = 0;
  uint32_t* ticket = nullptr;
};

// Brick decomposition of the Lorenzo kernels (one wave64 per brick).
struct LorenzoGeom {
  int ndim;
  int V;                  // elements per lane along x
  uint32_t nbx, nby, nbz; // bricks per axis
  uint32_t nbricks;
  uint32_t brick_elems;   // elements per full brick
};

LorenzoGeom lorenzo_geom(int ndim, size_t lx, size_t ly, size_t lz, int elem_bytes);

template <typename T>
int launch_lorenzo_c(const T* in, size_t lx, size_t ly, size_t lz, double eb, int radius, bool zigzag,
                     const LorenzoGeom& g, uint16_t* codes, const OutlierSink& ol, uint32_t* hist,
                     int bklen, hipStream_t st, const HostPub& pub = HostPub{});

// 1-D Lorenzo (non-ZigZag) reads the outlier values straight from the archive's cells when they
// are in strictly increasing index order (this compressor's archives without spill): code 0 marks
// exactly the outliers, so the k-th zero code of a brick takes the brick's k-th cell.  bstart
// (nbricks + 1) and the unsorted flag come from launch_x1d_bounds; an unsorted list falls back
// to the scatter (launch_scatter with only_if = unsorted) and reads from `out`.
struct X1dOutliers {
  const uint32_t* cells = nullptr;
  size_t ncell = 0;
  const uint32_t* bstart = nullptr;
  const uint32_t* unsorted = nullptr;  // == epoch: unsorted (the flag word is never reset)
  uint32_t epoch = 0;
};
// bstart over units of 2^ushift elements (16384: the 1-D reconstruction; 256: 1-D brick chunks)
int launch_x1d_bounds(const uint32_t* cells, size_t ncell, size_t n, uint32_t nbricks, uint32_t* bstart,
                      uint32_t* unsorted, uint32_t epoch, hipStream_t st, uint32_t ushift = 14);

template <typename T>
int launch_lorenzo_x(const uint16_t* codes, T* out, size_t lx, size_t ly, size_t lz, double eb, int radius,
                     bool zigzag, const LorenzoGeom& g, hipStream_t st, const X1dOutliers* ox = nullptr);

template <typename T>
int launch_scatter(const uint32_t* cells, size_t nnz, T* out, size_t n, hipStream_t st,
                   const uint32_t* only_if = nullptr, uint32_t epoch = 0);

// ---- Huffman (huffman.hip) ---------------------------------------------------------------
struct HfEncodeArgs {
  const uint16_t* codes;
  size_t n;
  const uint32_t* book;  // device u32[bklen]
  int bklen;
  int sublen;            // multiple of 256, <= 8192
  int pardeg;
  uint32_t* par_nbit;    // archive segment
  uint32_t* par_entry;   // archive segment
  uint32_t* bitstream;   // archive segment (4-byte aligned)
  unsigned long long* status;  // pardeg/kGroup+1 lookback words, zeroed before launch
  unsigned int* timeout;       // set nonzero if a bounded spin gave up
  uint32_t* temp;              // scratch of hf_encode_temp_words(); nullptr = look-back encoder
  unsigned long long* total_nbit = nullptr;  // if set (zeroed before): the tile-sum pass adds every chunk's bits
  uint32_t* ticket = nullptr;  // kPubTicketWords words zeroed per call: up to 2,048 tiles the tile-sum
                               // launch's last workgroup scans them (k_hf_tile_scan not launched)
};
int launch_hf_encode(const HfEncodeArgs& a, hipStream_t st);
size_t hf_encode_temp_words(int sublen, int pardeg);

// decode table scratch (u32 words): L1 4096 | maxl | first[] | bases | L2 2048, then a 32-B
// sink the lane decoder stores to when it has nothing to flush (HfDecodeArgs::lut)
constexpr int kHfDecTableWords = 4096 + 128 + 2048;
constexpr int kHfDecScratchWords = kHfDecTableWords + 16;

struct HfDecodeArgs {
  const uint32_t* bitstream;
  const uint8_t* revbook;  // first i32[32] | entry i32[32] | keys u16[bklen]
  int bklen;
  const uint32_t* par_nbit;
  const uint32_t* par_entry;
  int sublen;
  int pardeg;
  size_t n;
  uint16_t* out;
  uint32_t* lut;     // scratch u32[kHfDecTableWords], 16-B aligned (built by the decode launch)
  size_t avg_cells;  // average cells per chunk (sizes the LDS staging area); 0 = unknown
  int decoder;       // PSZ_AMD_DECODER_* (0 auto)
};
int launch_hf_decode(const HfDecodeArgs& a, hipStream_t st);

// ---- pipeline glue (pipeline_kernels.hip) ---------------------------------------------------
struct FinalizeArgs {
  // Huffman
  const uint32_t* par_nbit;
  const uint32_t* par_entry;
  int pardeg;
  // outliers
  const uint32_t* brick_cnt;
  uint32_t nbricks;
  uint32_t cap_per_brick;
  const uint32_t* spill_cnt;
  uint32_t spill_cap;
  uint32_t* brick_off;  // scratch u32[nbricks+1]
  CompressInfo* info;
  const uint32_t* spill_start = nullptr;  // OutlierSink::spill_start (ranged spill) or nullptr
  bool sizes_known = false;  // brick path: total_nbit / total_ncell already in info (reservation)
  bool nbit_known = false;   // info->total_nbit already summed (the encoder's tile-sum pass)
};
// psz_tpl / phf_tpl non-null: the same workgroup also writes both headers (no separate launch)
int launch_finalize_scan(const FinalizeArgs& a, hipStream_t st, const void* psz_tpl = nullptr,
                         const void* phf_tpl = nullptr, uint8_t* archive = nullptr, size_t phf_offset = 0,
                         size_t bitstream_rel = 0);

struct OutlierCopyArgs {
  const uint64_t* slots;
  const uint32_t* brick_cnt;
  const uint32_t* brick_off;
  uint32_t nbricks;
  uint32_t cap_per_brick;
  const uint64_t* spill;
  const uint32_t* spill_cnt;
  uint32_t spill_cap;
  const CompressInfo* info;
  uint8_t* archive;         // base of the archive
  size_t bitstream_offset;  // byte offset of the bitstream (outliers follow it)
  const uint32_t* spill_start = nullptr;  // OutlierSink::spill_start (ranged spill) or nullptr
};
int launch_outlier_copy(const OutlierCopyArgs& a, hipStream_t st, const HostPub& pub = HostPub{});


// small host<->device transfers through host-mapped pinned memory (no stream sync)
int launch_publish(const XferRegions& r, uint32_t* flag, uint32_t epoch, hipStream_t st);
int launch_upload(const XferRegions& r, hipStream_t st);
// upload behind a device-polled host gate (the host sets *gate = epoch when the data is ready)
int launch_gate_upload(const XferRegions& r, const uint32_t* gate, uint32_t epoch, unsigned int* timeout,
                       hipStream_t st);
int launch_zero(const XferRegions& r, hipStream_t st);  // dst/nwords only
// device codebook (book_device.hh): one workgroup, histogram (+ smooth per bin) -> book + revbook
int launch_book_device(const uint32_t* hist, int bklen, uint32_t smooth, uint32_t* book, uint8_t* revbook,
                       hipStream_t st);
int launch_excess(const uint32_t* spill_cnt, uint32_t cap, uint32_t* dst, hipStream_t st);

// ---- cuSZ-i spline3 (spline.hip) -----------------------------------------------------------
struct SplineGeom {
  uint32_t gdx, gdy, gdz, ntiles;  // 32 x 8 x 8 tiles (spline3.cu:29)
  size_t anchor_len;               // ceil(x/8) * ceil(y/8) * ceil(z/8) (buf_comp.cc:35-43)
};
SplineGeom spline_geom(size_t x, size_t y, size_t z);

template <typename T>
struct SplineArgs {
  const T* in;
  uint32_t X, Y, Z;
  uint32_t gdx, gdy, gdz, ntiles;
  float eb_r, ebx2;  // (float)(1/eb), (float)(2 eb): compressor.inl:107-108, FP = float
  int radius;
  int bklen;
  uint16_t* codes;
  T* anchor;      // anchor_len values (written into the archive's anchor segment)
  OutlierSink ol; // one slot range per tile (cap_per_brick), spill list beyond
  uint32_t* hist;
};
template <typename T>
int launch_spline3_c(const SplineArgs<T>& a, hipStream_t st);

template <typename T>
struct SplineXArgs {
  const uint16_t* codes;
  const T* anchor;
  T* out;
  uint32_t X, Y, Z;
  uint32_t gdx, gdy, gdz, ntiles;
  float eb_r, ebx2;
  int radius;
  const uint32_t* boff = nullptr;     // per-tile bucket offsets (set by the launcher)
  const uint32_t* bucket = nullptr;   // outlier cells {code bits, idx} grouped by tile (unsorted archives)
  const uint32_t* cells = nullptr;    // the archive's cells (already grouped: archives of this compressor)
  const uint32_t* unsorted = nullptr; // device flag: use `bucket` instead of `cells`
  size_t nbucket = 0;
  // outlier index -> (x, y, z) by multiply-high: q = mulhi(i, m) >> s for divisors X and Y
  // (set by the launcher; exact for i < 2^31; ndiv = true makes the kernel divide instead)
  uint32_t mX = 0, sX = 0, mY = 0, sY = 0;
  bool ndiv = true;
};
// cells: the archive's outlier segment ({f32 code, u32 idx} each); scratch: spline_x_scratch_words
template <typename T>
int launch_spline3_x(SplineXArgs<T> a, const uint32_t* cells, size_t ncell, uint32_t* scratch, hipStream_t st);
size_t spline_x_scratch_words(uint32_t ntiles, size_t ncell);

// ---- fused brick pipeline (brick.hip) --------------------------------------------------------
// A wave owns a W x 8 x 8 brick (W = 64 V); the Huffman chunk length equals W so each brick row
// is one chunk.  Eligible: 3-D with lx % W == 0, and 1-D (a brick = 64 consecutive chunks, 16
// tiles of 1024; the last brick and chunk may be short).
struct BrickGeom {
  bool ok;
  int ndim;
  int V, W;
  uint32_t nbx, nby, nbz, nbricks;
  uint32_t brick_elems;
  uint32_t nchunks;
  size_t n;
};
BrickGeom brick_geom(int ndim, size_t lx, size_t ly, size_t lz, int elem_bytes);

struct BrickLaunch {
  BrickGeom g;
  uint32_t lx, ly, lz;
  int grid_scan, grid_pack;  // workgroups of the encode passes (per-device occupancy)
  int ncu;
};

// fills ncu and the encode-pass grids for `device`
int brick_configure(BrickLaunch& L, int elem_bytes, int device);

// The codebook sample inside pass 1 (sampled codebook mode): every `stride`-th brick (offset
// stride / 2) is visited FIRST -- iteration j < count takes sample brick j -- and adds its
// histogram to hist (u32[bklen], global atomics); then done (a u32) counts it, and the wave that
// completes the sample publishes it to the host (pub_dst, then *pub_flag = pub_epoch), which
// builds the codebook while pass 1 goes on.  hist == nullptr: no sample, bricks in index order.
// the sample histogram's bins lie a 64-B line apart: the sample bricks finish together (first
// round of pass 1) and their atomics would otherwise queue on the one or two memory channels of
// a dense 4 KB array (measured: pass 1 +60 us)
constexpr int kSampleBinStride = 16;
struct BrickSample {
  uint32_t* hist = nullptr;  // u32[kMaxBklen * kSampleBinStride]
  uint32_t* done = nullptr;
  uint32_t stride = 1, count = 0;
  uint32_t* pub_dst = nullptr;   // host-mapped u32[bklen]
  uint32_t* pub_flag = nullptr;  // host-mapped
  uint32_t pub_epoch = 0;
  int bklen = 0;
};
BrickSample brick_sample_plan(uint32_t nbricks, uint32_t* hist, uint32_t* done);


// Quant codes between the two encode passes, in brick order (row r of brick b at (64 b + r) W).
// A row whose codes all lie in [c0, c0 + 254] or are 0 (outliers) is stored as bytes (code - c0;
// 255 for code 0) in c8; any other
// row as u16 codes in c16, with bit r of rowmask[b] set.  c0 = radius - 127 (ZigZag: 0): the
// rows that are not u16 are about 90 % of a smooth field's (those off the tiles' first z plane).
struct BrickCodes {
  uint16_t* c16;      // nbricks * 64 * W u16 (written only for the u16 rows)
  uint8_t* c8;        // nbricks * 64 * W bytes
  uint64_t* rowmask;  // nbricks
  uint32_t c0;
};
// pass 1: predict -> global + per-brick histograms, outliers, codes in brick order
template <typename T>
int launch_brick_scan(const BrickLaunch& L, const T* in, double eb, int radius, bool zz, const BrickSample& sample,
                      const OutlierSink& ol,
                      uint32_t* hist, uint16_t* bhist, const BrickCodes& bc, int bklen, hipStream_t st,
                      const HostPub& pub = HostPub{});
// archive plan (brick.hip k_brick_plan): region sizes, cell / outlier offsets, totals, headers
struct BrickPlanArgs {
  const uint16_t* bhist;  // per-brick histograms, stride brick_hist_stride(bklen)
  int bklen, bhs;
  const uint32_t* book;
  uint32_t nbricks, nunits, nbx, nby, ly, lz;  // units of brick_units(): regions, slots, histograms
  const uint32_t* brick_cnt;  // outliers per unit (pass 1)
  uint32_t cap_per_brick;     // outlier slot capacity per unit
  const uint64_t* slots;      // per-unit outlier slots
  const uint64_t* spill;
  const uint32_t* spill_cnt;
  uint32_t spill_cap;
  uint32_t nblk;              // plan blocks = brick_plan_blocks(nbricks)
  uint32_t* ub;               // per brick: region cells
  uint32_t* cell_local;       // per brick: cell offset inside its plan block
  uint32_t* ol_local;         // per brick: outlier offset inside its plan block
  uint32_t* cell_pre;         // nblk + 1: block prefixes, [nblk] = total cells
  uint32_t* ol_pre;           // nblk + 1: block prefixes, [nblk] = slot outliers
  CompressInfo* info;         // totals
  uint8_t* archive;
  size_t phf_offset, bitstream_rel;
  uint32_t nd = 3;       // 1: 1-D bricks (64 consecutive chunks; the last chunk may be short)
  uint32_t nchunks = 0;  // 1-D: chunks of the field
  size_t n = 0;          // 1-D: elements of the field
  uint32_t* ticket = nullptr;  // 9 words zeroed per call: the two-level last-block ticket
};
uint32_t brick_units(uint32_t nbricks);
uint32_t brick_plan_blocks(uint32_t nbricks);
int brick_hist_stride(int bklen);
int launch_brick_plan(const BrickLaunch& L, const BrickPlanArgs& a, const void* psz_tpl, const void* phf_tpl,
                      hipStream_t st);
// pass 2: brick-ordered codes -> Huffman cells at each brick's reserved region
int launch_brick_pack(const BrickLaunch& L, const BrickCodes& bc, const uint32_t* book, int bklen,
                      const BrickPlanArgs& plan, uint32_t* par_nbit, uint32_t* par_entry, uint32_t* bitstream,
                      int reverse, unsigned int* overflow, hipStream_t st, const HostPub& pub = HostPub{});
struct BrickSingle {
  OutlierSink ol;              // one slot per (brick, y-step): cap_per_brick = the slot's cap
  uint32_t* book;              // device book (the stream kernel's workgroup 0 writes it)
  int bklen;
  uint32_t *par_nbit, *par_entry, *bitstream;
  uint32_t bs_cap;             // bitstream capacity (cells)
  unsigned long long* status;  // nbricks words, zeroed per call
  uint32_t* ticket;            // zeroed per call
  uint32_t* ol_dst;            // per slot: its first cell in the archive's outlier segment
  CompressInfo* info;          // zeroed per call
  unsigned int* timeout;
  uint8_t* archive;
  size_t phf_offset, bits_rel;
  const uint32_t* gate;        // host-mapped: reaches gate_epoch once the host's book is written
  uint32_t gate_epoch;
  const uint32_t* h_book;      // host-mapped book and reverse book
  const uint32_t* h_revbook;
  uint32_t* revbook;           // the archive's reverse book
  int rv_words;
  uint32_t* book_flag;         // device word (never reset)
};
// single-pass mode (brick.hip): the sample histogram into hist (u32[kMaxBklen * kSampleBinStride],
// zeroed; bins one line apart); its last workgroup (ticket: kPubTicketWords words, zeroed) copies
// it to the host-mapped h_hist and sets *flag = epoch; the host builds the codebook.  Then the
// streaming pass, which takes the host's book behind a device-polled gate (+ finish: outlier
// segment, headers, the compress summary)
template <typename T>
int launch_brick_sample(const BrickLaunch& L, const T* in, double eb, int radius, bool zz, uint32_t* hist, int bklen,
                        uint32_t* ticket, uint32_t* h_hist, uint32_t* flag, uint32_t epoch, hipStream_t st);
template <typename T>
int launch_brick_stream(const BrickLaunch& L, const T* in, double eb, int radius, bool zz, const BrickSingle& s,
                        const void* psz_tpl, const void* phf_tpl, hipStream_t st, const HostPub& pub);
// Outlier cells for the fused decoder: when the archive's cells are grouped by brick and sorted
// by (row, x) (k_brick_cell_bounds checks; this compressor writes them so), the decoder ranks the
// zero codes of each row against the brick's cells and no scatter pass is needed; otherwise
// (*unsorted set) the scatter pass has written the values into `out`, which the decoder reads.
struct BrickOutliers {
  const uint32_t* cells = nullptr;  // archive cells {f32 value, u32 idx}
  size_t ncell = 0;
  const uint32_t* bstart = nullptr;   // nbricks + 1
  const uint32_t* unsorted = nullptr;  // == epoch: unsorted (the flag word is never reset)
  uint32_t epoch = 0;
};
int launch_brick_cell_bounds(const BrickLaunch& L, const uint32_t* cells, size_t ncell, uint32_t* bstart,
                             uint32_t* unsorted, uint32_t epoch, hipStream_t st);
// decode only, any archive whose chunk length is a multiple of 64: chunk c's codes to
// codes[sublen c ...] (index order)
int launch_chunk_decode(const BrickLaunch& L, const uint32_t* bitstream, size_t bs_words, const uint8_t* revbook,
                        int bklen, const uint32_t* par_nbit, const uint32_t* par_entry, uint16_t* codes, size_t n,
                        uint32_t nchunks, uint32_t sublen, hipStream_t st);
template <typename T>
int launch_brick_decode(const BrickLaunch& L, const uint32_t* bitstream, size_t bs_words, const uint8_t* revbook,
                        int bklen, const uint32_t* par_nbit, const uint32_t* par_entry, T* out, double eb, int radius,
                        bool zz, const BrickOutliers& ol, hipStream_t st);

// min / max (Rel mode, extrema.cuhip.inl:86-208), writes {min, max} as doubles
template <typename T>
int launch_extrema(const T* in, size_t n, double* d_minmax, unsigned int* d_scratch, hipStream_t st);

}  // namespace cusz_amd
