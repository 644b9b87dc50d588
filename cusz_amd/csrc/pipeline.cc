// cusz_amd/csrc/pipeline.cc -- the compression pipeline behind the cuSZ C API.
//
// Replaces psz::compression_pipeline<T,u2> (psz/src/compressor.inl:268-529) and the C-API
// glue of psz/src/libcusz.cc:219-366.  One device-resident Pipeline per psz_resource:
//
//   compress:  [extrema (Rel)] -> predict+quantize+histogram+outliers (1 kernel)
//              -> histogram D2H, host codebook, book/revbook H2D (the one host round trip
//                 the reference algorithm needs: the codebook depends on the full histogram)
//              -> Huffman encode straight into the archive (1 kernel, device look-back)
//              -> finalize: outlier compaction + headers written on device
//              -> one 176-B header read-back (compress is synchronous, as in the reference)
//   decompress: outlier scatter -> Huffman decode -> Lorenzo reconstruct (queued, no sync)
//
// The reference does 5+ host round trips per compress and copies a 2N-byte buffer
// (SURVEY.md §3.1); here the archive is assembled in place.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <tuple>

#include "common.hh"
#include "cusz.h"
#include "cusz_amd.h"
#include "cusz_rev1.h"
#include "hf.h"
#include "kernels.hh"

namespace cusz_amd {

int build_codebook(const uint32_t* hist, int bklen, uint32_t* book, uint8_t* revbook);
int build_codebook_twoqueue(const uint32_t* hist, int bklen, uint32_t smooth, uint32_t* book, uint8_t* revbook);
int hf_encode_groups(int sublen, int pardeg);
size_t hf_encode_temp_words(int sublen, int pardeg);

int report_hip_error(hipError_t e, const char* expr, const char* file, int line)
{
  std::fprintf(stderr, "[cusz_amd] HIP error %d (%s) at %s:%d: %s\n", (int)e, hipGetErrorString(e), file, line,
               expr);
  return PSZ_AMD_ERR_DEVICE;
}

static int ndim_of(psz_len l)
{  // launch.hh:19-28
  if (l.z == 1 && l.y == 1) return 1;
  if (l.z == 1) return 2;
  return 3;
}

// Chunk length (vle_sublen).  The reference sizes chunks for one encode thread per chunk on
// maxThreadsPerBlock * nSM / 4 threads (libphf.cc:26-70, which notes "ROCm GPUs should use
// different constants").  Here the decoder is the consumer that needs the parallelism: one lane
// per chunk, two waves per SIMD -> nCU * 4 SIMDs * 64 lanes * 2 chunks (131,072 on MI355X, so
// 512^3 gets sublen 1024, the reference's own HFR setting, hf_buf.cc:77).  Multiple of 256,
// at most 8192 (encoder LDS); any value is readable by either decoder.
static void tune_chunking(size_t n, int device, int* sublen, int* pardeg)
{
  int ncu = 256;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || ncu < 1) ncu = 256;
  const size_t lanes = (size_t)ncu * 4 * 64 * 2;
  size_t s = (std::max<size_t>(n, 1) - 1) / lanes + 1;
  s = ((s - 1) / 256 + 1) * 256;
  if (s > 8192) s = 8192;
  *sublen = (int)s;
  *pardeg = (int)((std::max<size_t>(n, 1) - 1) / s + 1);
}

struct Pipeline {
  psz_dtype dtype;
  psz_len len;
  size_t n = 0;
  int ndim = 1;
  int device = 0;
  hipStream_t stream = nullptr;
  int elem_bytes = 4;

  LorenzoGeom geom{};
  BrickLaunch bl{};               // fused brick path (brick.hip); bl.g.ok when eligible
  int layout = 0;                 // PSZ_AMD_LAYOUT_*: 0 brick layout when eligible, 1 reference layout
  bool layout_set = false;        // PSZ_AMD_LAYOUT_BRICK_FORCE: bricks also for small 2-D fields
  int codebook = PSZ_AMD_CODEBOOK_SAMPLED;  // PSZ_AMD_CODEBOOK_*: sampled device book (default),
                                            // reference book (exact), streaming single pass
  uint32_t* d_shist = nullptr;    // pass 1's codebook sample: strided histogram + counter
  uint16_t* d_bhist = nullptr;    // per-brick u16 histograms (pass 1 -> reservation)
  uint32_t* d_ub = nullptr;       // per-brick region upper bounds (cells)
  uint32_t* d_bbase = nullptr;    // per-brick cell offsets inside their plan block
  uint32_t* d_plan = nullptr;     // plan block prefixes: cells | outliers (nblk + 1 each)
  SplineGeom sgeom{};
  uint32_t spl_cap = 0;           // outlier slots per spline tile
  size_t spl_slot_cells = 0;      // capacity of the spline slot area (allocated on first use)
  uint64_t* d_spl_slots = nullptr;
  uint32_t* d_spl_cnt = nullptr;  // per-tile outlier counts | offsets
  uint32_t* d_spl_off = nullptr;
  uint32_t* d_spl_sps = nullptr;  // per-tile spill range starts
  uint32_t* d_spl_x = nullptr;    // decompression buckets
  uint32_t* d_x1d = nullptr;      // 1-D decompression: per-brick first outlier cell + unsorted flag
  uint32_t cell_epoch = 0;        // tags the unsorted flag of the current decompress (never 0)
  uint32_t next_cell_epoch() { return cell_epoch = cell_epoch + 1 ? cell_epoch + 1 : 1; }
  size_t spl_x_words = 0;
  int sublen = 256, pardeg = 1;
  int user_sublen = 0;
  int tuned_sublen = 256;  // tune_chunking's choice for this field
  int decoder = 0;  // PSZ_AMD_DECODER_*
  int last_layout = 1;   // layout of the last compress (PSZ_AMD_LAYOUT_*)
  int pack_reverse = 1;  // pass 2 walks bricks last-to-first (reuses pass 1's cache tail)
  uint32_t cap_per_brick = 0, spill_cap = 0;
  size_t splen = 0;

  // device
  uint16_t* d_codes = nullptr;
  uint8_t* d_codes8 = nullptr;     // brick layout: byte rows between the encode passes
  uint64_t* d_rowmask = nullptr;   // brick layout: u16 rows per brick
  uint32_t* d_hist = nullptr;
  uint32_t* d_book = nullptr;
  uint64_t* d_slots = nullptr;
  uint32_t* d_brick_cnt = nullptr;
  uint32_t* d_brick_off = nullptr;
  uint64_t* d_spill = nullptr;
  uint8_t* d_small = nullptr;  // spill_cnt | timeout | info | minmax | extrema scratch
  unsigned long long* d_status = nullptr;
  uint32_t* d_enc_temp = nullptr;  // encoder scratch (chunk cells at a worst-case stride)
  size_t status_words = 0;
  uint8_t* d_archive = nullptr;
  size_t archive_cap = 0;

  // pinned, host-mapped, coherent transfer area (kernels write it, the host polls flags)
  uint8_t* h_xfer = nullptr;
  uint32_t epoch = 0;
  uint32_t gate_epoch = 0;       // host -> stream gate (flag 5): the upload kernel polls it
  uint32_t summary_epoch = 0;    // != 0: the compress summary is published by the pack kernel
  bool gate = true;              // brick encode queued behind a device-polled host gate (flag 5)
  static constexpr size_t kXferBytes = 16384;
  volatile uint32_t* flag(int i) { return reinterpret_cast<volatile uint32_t*>(h_xfer) + i; }  // 0..15
  uint32_t* h_hist() { return reinterpret_cast<uint32_t*>(h_xfer + 64); }               // 4 KB
  uint32_t* h_book() { return reinterpret_cast<uint32_t*>(h_xfer + 64 + 4096); }        // 4 KB
  uint8_t* h_revbook() { return h_xfer + 64 + 8192; }                                    // 2304 B
  uint8_t* h_readback() const { return h_xfer + 64 + 8192 + 2560; }                            // 1 KB

  bool timing = false;
  bool broken = false;  // an allocation failed mid-call (grow_spill): every later compress fails
  hipEvent_t ev[12] = {};
  float stage_ms[PSZ_AMD_T_COUNT] = {0};

  uint32_t* spill_cnt() { return reinterpret_cast<uint32_t*>(d_small); }
  unsigned int* timeout() { return reinterpret_cast<unsigned int*>(d_small + 16); }
  CompressInfo* info() { return reinterpret_cast<CompressInfo*>(d_small + 64); }
  double* minmax() { return reinterpret_cast<double*>(d_small + 256); }
  unsigned int* ext_scratch() { return reinterpret_cast<unsigned int*>(d_small + 512); }
  uint32_t* dec_lut() { return reinterpret_cast<uint32_t*>(d_small + 512 + 2 * 1024 * 8); }
  static constexpr size_t kSmallBytes = 512 + 2 * 1024 * 8 + kHfDecScratchWords * 4;
  // the publish tickets (9 words each, pub_device.hh); bytes [0, kSmallZeroBytes) are zeroed
  // at the start of every compress
  uint32_t* hist_ticket() { return reinterpret_cast<uint32_t*>(d_small + 160); }
  uint32_t* summary_ticket() { return reinterpret_cast<uint32_t*>(d_small + 196); }
  uint32_t* plan_ticket() { return reinterpret_cast<uint32_t*>(d_small + 112); }
  // the single-pass mode's codebook flag (brick.hip k_brick3_stream): never zeroed, epoch-compared
  uint32_t* book_flag() { return reinterpret_cast<uint32_t*>(d_small + 240); }
  static constexpr uint32_t kStreamSlots = 8;  // outlier slots per brick in the single-pass mode (one per y-step)
  static constexpr size_t kSmallZeroBytes = 232;
  static_assert(64 + sizeof(CompressInfo) <= 112 && 112 + 36 <= 160 && 196 + 36 <= kSmallZeroBytes &&
                    kSmallZeroBytes <= 256,
                "small-buffer layout");

  ~Pipeline() { release(); }

  void release()
  {
    if (d_shist) (void)hipFree(d_shist), d_shist = nullptr;
    for (void* p : {(void*)d_codes, (void*)d_hist, (void*)d_book, (void*)d_slots, (void*)d_brick_cnt,
                    (void*)d_brick_off, (void*)d_spill, (void*)d_small, (void*)d_status, (void*)d_archive,
                    (void*)d_enc_temp, (void*)d_spl_slots, (void*)d_spl_cnt, (void*)d_spl_off, (void*)d_spl_x, (void*)d_spl_sps,
                    (void*)d_bhist, (void*)d_ub, (void*)d_bbase, (void*)d_plan, (void*)d_x1d, (void*)d_codes8,
                    (void*)d_rowmask})
      if (p) (void)hipFree(p);
    if (h_xfer) (void)hipHostFree(h_xfer);
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e), e = nullptr;
    d_codes = nullptr, d_hist = nullptr, d_book = nullptr, d_slots = nullptr, d_brick_cnt = nullptr;
    d_brick_off = nullptr, d_spill = nullptr, d_small = nullptr, d_status = nullptr, d_archive = nullptr;
    d_enc_temp = nullptr;
    d_bhist = nullptr, d_ub = nullptr, d_bbase = nullptr, d_plan = nullptr, d_x1d = nullptr;
    d_codes8 = nullptr, d_rowmask = nullptr;
    d_spl_slots = nullptr, d_spl_cnt = nullptr, d_spl_off = nullptr, d_spl_x = nullptr, d_spl_sps = nullptr;
    spl_slot_cells = 0, spl_x_words = 0;
    h_xfer = nullptr;
  }

  size_t rvbk_bytes(int bklen) const { return 4 * 64 + 2 * (size_t)bklen; }
  // outlier slot per brick unit (brick.hip kUnitBricks bricks): 10 % of its elements + 16 at
  // first; a compress whose bricks spill grows it to the largest brick's count (grow_slots)
  uint32_t brick_slot_cap = 0;
  uint32_t brick_cap() const { return brick_slot_cap; }
  uint32_t brick_unit_elems() const
  {
    const uint32_t nu = brick_units(bl.g.nbricks), per = (bl.g.nbricks + nu - 1) / nu;
    return bl.g.brick_elems * per;
  }
  // cells of every slot (reference-layout bricks and brick-layout units share d_slots)
  size_t slot_cells_total() const
  {
    size_t c = (size_t)geom.nbricks * cap_per_brick;
    if (bl.g.ok) c = std::max(c, (size_t)brick_units(bl.g.nbricks) * brick_slot_cap);
    return c;
  }
  int grow_events = 0;  // capacity growths (a compress that warned repeats only after one)

  // fused brick path: 3-D, eligible shape, Lorenzo, default chunking (chunk = brick row)
  bool use_brick(psz_predictor pred) const
  {
    // 2-D linear bricks by default only when there are enough to fill the device (a wave walks a
    // brick serially: 3600 x 1800 has 396, the reference layout is faster there)
    const bool enough = bl.g.ndim != 2 || layout_set || bl.g.nbricks >= 4u * (uint32_t)bl.ncu;
    return bl.g.ok && layout == 0 && enough && (pred == Lorenzo || pred == LorenzoZigZag) &&
           (user_sublen == 0 || user_sublen == bl.g.W);
  }

  size_t bitstream_cells_cap() const { return (n * kLmax + 31) / 32 + (size_t)pardeg + 8; }

  int init(psz_dtype dt, psz_len l, void* st)
  {
    dtype = dt;
    len = l;
    if (l.x == 0 || l.y == 0 || l.z == 0) return PSZ_ABORT_UNSUPPORTED_DIMENSION;
    n = l.x * l.y * l.z;
    if (n >= (1ull << 32)) return PSZ_ABORT_UNSUPPORTED_DIMENSION;  // u32 outlier index (sp_interface.h)
    ndim = ndim_of(l);
    elem_bytes = dt == F8 ? 8 : 4;
    // the 2-D Lorenzo kernels address one row through a 32-bit buffer range: a row of 2 GiB or
    // more is a shape this build does not take (creation fails with this status; the caller
    // reshapes such a field to 1-D)
    if (ndim == 2 && l.x * (size_t)elem_bytes >= 0x80000000ull) return PSZ_ABORT_UNSUPPORTED_DIMENSION;
    stream = (hipStream_t)st;
    CUSZ_AMD_HIP_CHECK(hipGetDevice(&device));
    tune_chunking(n, device, &sublen, &pardeg);
    tuned_sublen = sublen;
    geom = lorenzo_geom(ndim, l.x, l.y, l.z, elem_bytes);
    if (ndim == 1) {
      // per-unit first cell + unsorted word: units of 16384 (reconstruction) or 256 (brick chunks)
      const size_t units = std::max<size_t>(geom.nbricks, (n + 255) / 256);
      CUSZ_AMD_HIP_CHECK(hipMalloc(&d_x1d, (units + 2) * 4));
      CUSZ_AMD_HIP_CHECK(hipMemset(d_x1d, 0, (units + 2) * 4));  // unsorted word: no epoch yet
    }
    sgeom = spline_geom(l.x, l.y, l.z);
    spl_cap = (uint32_t)(std::min<size_t>(l.x, 32) * std::min<size_t>(l.y, 8) * std::min<size_t>(l.z, 8) / 10 + 16);
    // outlier capacity: 10 % of the input like the reference (buf_comp.hh:55), as per-brick
    // slots plus an equally large spill list for bricks above 10 %.
    cap_per_brick = geom.brick_elems / 10 + 16;
    spill_cap = (uint32_t)(n / 10 + 1024);
    bl.g = brick_geom(ndim, l.x, l.y, l.z, elem_bytes);
    bl.lx = (uint32_t)l.x, bl.ly = (uint32_t)l.y, bl.lz = (uint32_t)l.z;
    uint32_t max_bricks = geom.nbricks;
    if (bl.g.ok) {
      CUSZ_AMD_HIP_CHECK((hipError_t)brick_configure(bl, elem_bytes, device));
      brick_slot_cap = brick_unit_elems() / 10 + 16;
      max_bricks = std::max(max_bricks, bl.g.nbricks);
      CUSZ_AMD_HIP_CHECK(hipMalloc(&d_bhist, (size_t)bl.g.nbricks * kMaxBklen * sizeof(uint16_t)));
      CUSZ_AMD_HIP_CHECK(hipMalloc(&d_ub, (size_t)bl.g.nbricks * 4));
      CUSZ_AMD_HIP_CHECK(hipMalloc(&d_bbase, ((size_t)bl.g.nbricks + 1) * 4));
      CUSZ_AMD_HIP_CHECK(hipMalloc(&d_plan, 2 * ((size_t)brick_plan_blocks(bl.g.nbricks) + 1) * 4));
      // fused decompression: per-brick first outlier cell + unsorted flag (d_x1d's role in 1-D)
      if (!d_x1d) {
        CUSZ_AMD_HIP_CHECK(hipMalloc(&d_x1d, ((size_t)bl.g.nbricks + 2) * 4));
        CUSZ_AMD_HIP_CHECK(hipMemset(d_x1d, 0, ((size_t)bl.g.nbricks + 2) * 4));
      }
      CUSZ_AMD_HIP_CHECK(hipMalloc(&d_codes8, (size_t)bl.g.nbricks * bl.g.brick_elems + 64));  // + 8-B load slack
      CUSZ_AMD_HIP_CHECK(hipMalloc(&d_rowmask, (size_t)bl.g.nbricks * 8));
    }

    // codes: index order (reference layout) or brick order (brick layout: whole bricks)
    const size_t code_len = std::max(n + 64, bl.g.ok ? (size_t)bl.g.nbricks * bl.g.brick_elems : 0);
    CUSZ_AMD_HIP_CHECK(hipMalloc(&d_codes, code_len * sizeof(uint16_t)));
    CUSZ_AMD_HIP_CHECK(hipMalloc(&d_hist, (kMaxBklen + 4) * sizeof(uint32_t)));  // + the sharded overflow word
    CUSZ_AMD_HIP_CHECK(hipMalloc(&d_book, kMaxBklen * sizeof(uint32_t)));
    CUSZ_AMD_HIP_CHECK(hipMalloc(&d_slots, slot_cells_total() * 8));
    CUSZ_AMD_HIP_CHECK(hipMalloc(&d_brick_cnt, (size_t)max_bricks * 4));
    CUSZ_AMD_HIP_CHECK(hipMalloc(&d_brick_off, ((size_t)max_bricks + 1) * 4));
    CUSZ_AMD_HIP_CHECK(hipMalloc(&d_spill, (size_t)spill_cap * 8));
    CUSZ_AMD_HIP_CHECK(hipMalloc(&d_small, kSmallBytes));
    CUSZ_AMD_HIP_CHECK(hipMemset(d_small, 0, kSmallBytes));
    CUSZ_AMD_HIP_CHECK(alloc_chunk_state());
    CUSZ_AMD_HIP_CHECK(hipHostMalloc(&h_xfer, kXferBytes, hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(h_xfer, 0, kXferBytes);
    for (auto& e : ev) CUSZ_AMD_HIP_CHECK(hipEventCreate(&e));
    if (bl.g.ok)  // pass 1's sample: strided histogram + the done counter
      CUSZ_AMD_HIP_CHECK(hipMalloc(&d_shist, ((size_t)kMaxBklen * kSampleBinStride + 16) * sizeof(uint32_t)));
    if (const char* g = getenv("CUSZ_AMD_NO_GATE")) gate = atoi(g) == 0;
    return PSZ_SUCCESS;
  }

  // Outlier capacity beyond the reference's 10 % (buf_comp.cc:87-88, compressor.inl:368-372 fail
  // the compress there): a spill list for `need` cells (bounded by n) and an archive to match.
  // 1: grown, 0: already at the bound, -1: allocation failure.
  int grow_spill(uint64_t need)
  {
    const uint64_t cap = std::min<uint64_t>(need + need / 8 + 1024, (uint64_t)n + 1024);
    if (cap <= spill_cap) return 0;
    // the new list is allocated before the old one is freed; on any failure the manager is marked
    // broken (every later compress returns PSZ_AMD_ERR_DEVICE instead of handing a kernel a null
    // list or archive)
    uint64_t* grown = nullptr;
    if (hipMalloc(&grown, cap * 8) != hipSuccess) {
      broken = true;
      return -1;
    }
    (void)hipFree(d_spill);
    d_spill = grown;
    spill_cap = (uint32_t)cap;
    if (alloc_chunk_state() != hipSuccess) {
      broken = true;
      return -1;
    }
    grow_events++;
    return 1;
  }

  // Bricks with more outliers than their slot spilled to the shared list (archive valid, but the
  // list's order depends on the atomics, so the archive is not deterministic and the decoders
  // take the scatter path).  The slots of the layout just used grow to the largest brick's count
  // (bounded by the brick's elements) and the caller repeats: identical below the 10 % slots.
  // 1: grown, 0: already at the bound, -1: allocation failure (manager marked broken).
  int grow_slots(uint32_t need)
  {
    const bool brick = last_layout == PSZ_AMD_LAYOUT_BRICK;
    uint32_t& cap = brick ? brick_slot_cap : cap_per_brick;
    const uint32_t lim = brick ? brick_unit_elems() : geom.brick_elems;
    const uint32_t want = (uint32_t)std::min<uint64_t>(lim, (uint64_t)need + need / 8 + 16);
    if (want <= cap) return 0;
    cap = want;
    uint64_t* grown = nullptr;
    if (hipMalloc(&grown, slot_cells_total() * 8) != hipSuccess) {
      broken = true;
      return -1;
    }
    (void)hipFree(d_slots);
    d_slots = grown;
    if (alloc_chunk_state() != hipSuccess) {
      broken = true;
      return -1;
    }
    grow_events++;
    return 1;
  }

  hipError_t alloc_chunk_state()
  {
    if (d_status) (void)hipFree(d_status), d_status = nullptr;
    if (d_enc_temp) (void)hipFree(d_enc_temp), d_enc_temp = nullptr;
    if (const size_t tw = hf_encode_temp_words(sublen, pardeg)) {
      const hipError_t et = hipMalloc(&d_enc_temp, tw * 4);
      if (et != hipSuccess) return et;
    }
    if (d_archive) (void)hipFree(d_archive), d_archive = nullptr;
    status_words = (size_t)hf_encode_groups(sublen, pardeg) + 1;
    hipError_t e = hipMalloc(&d_status, status_words * 8);
    if (e != hipSuccess) return e;
    const size_t ol_cells = std::max(slot_cells_total(), (size_t)sgeom.ntiles * spl_cap);
    // chunk tables: the tuned chunking's, or the brick layout's (one chunk per brick row)
    const size_t chunks = std::max((size_t)pardeg, bl.g.ok ? (size_t)bl.g.nchunks : 0);
    archive_cap = 176 + (size_t)elem_bytes * sgeom.anchor_len + 128 + rvbk_bytes(kMaxBklen) + 8 * chunks +
                  4 * (bitstream_cells_cap() + chunks) + 8 * (ol_cells + spill_cap) + 64;
    return hipMalloc(&d_archive, archive_cap);
  }

  // device words -> host-mapped memory, then wait for the flag (fallback: stream sync)
  int fetch(XferRegions r, int fl)
  {
    const uint32_t e = ++epoch;
    CUSZ_AMD_HIP_CHECK((hipError_t)launch_publish(r, const_cast<uint32_t*>(flag(fl)), e, stream));
    return wait_flag(fl, e);
  }

  int wait_flag(int fl, uint32_t e)
  {
    for (long spin = 0;; spin++) {
      if (__atomic_load_n(flag(fl), __ATOMIC_ACQUIRE) == e) return PSZ_SUCCESS;
      if (spin > (1L << 26)) break;  // ~seconds: something is wrong, surface it via the runtime
      __builtin_ia32_pause();
    }
    CUSZ_AMD_HIP_CHECK(hipStreamSynchronize(stream));
    return __atomic_load_n(flag(fl), __ATOMIC_ACQUIRE) == e ? PSZ_SUCCESS : PSZ_AMD_ERR_DEVICE;
  }

  static XferRegions regions(std::initializer_list<std::tuple<void*, const void*, size_t>> l)
  {
    XferRegions r{};
    for (auto& [d, s, bytes] : l) {
      r.dst[r.count] = (uint32_t*)d;
      r.src[r.count] = (const uint32_t*)s;
      r.nwords[r.count] = (int)((bytes + 3) / 4);
      r.count++;
    }
    return r;
  }

  void mark(int i)
  {
    if (timing) (void)hipEventRecord(ev[i], stream);
  }

  float span(int a, int b)
  {
    float ms = 0;
    if (hipEventElapsedTime(&ms, ev[a], ev[b]) != hipSuccess) ms = -1;
    return ms;
  }

  // state carried from compress_scan (pass 1) to compress_finish (codebook onwards)
  struct Pending {
    bool active = false, brick = false, spl = false, zz = false;
    int radius = 0;
    uint32_t hist_epoch = 0;  // != 0: the scan published d_hist to h_hist() with this epoch (flag 2)
    bool ext = false;         // finish with a caller's (reduced) histogram + overflow word
    bool side_book = false;   // pass 1 publishes a codebook sample to the host (epoch: hist_epoch)
    size_t anchor_bytes = 0;
  } pend;

  template <typename T>
  int compress(psz_header* h, const T* in, uint8_t** out, size_t* outlen)
  {
    if (broken) return PSZ_AMD_ERR_DEVICE;
    const psz_rc2 rc = h->rc;  // Rel mode scales eb in place: a second run starts from the caller's
    for (int run = 0;; run++) {
      const int g0 = grow_events;
      int s;
      if (codebook == PSZ_AMD_CODEBOOK_STREAM && bl.g.ndim == 3 && use_brick(h->pipeline.predictor))
        s = compress_sampled<T>(h, in, out, outlen);
      else {
        s = compress_scan<T>(h, in, true);
        if (!s) s = compress_finish(h, nullptr, out, outlen);
      }
      // bricks spilled past their slots (or past the spill list): the capacity has grown to hold
      // them, compress again (identical below the reference's 10 % cap, where this never runs)
      if (s != PSZ_WARN_OUTLIER_TOO_MANY || grow_events == g0 || run > 1) return s;
      h->rc = rc;
    }
  }

  // Pass 1: [extrema] -> predict + histogram + outliers (+ codes).  The histogram stays on the
  // device (d_hist) for compress_finish, or for a caller that reduces it across slabs first.
  // pub_hist: the brick scan publishes the histogram to the host itself (its last workgroup), for a
  // finish that follows with the scan's own histogram
  template <typename T>
  int compress_scan(psz_header* h, const T* in, bool pub_hist = false)
  {
    if (broken) return PSZ_AMD_ERR_DEVICE;
    pend.active = false;
    pend.ext = false;
    pend.side_book = false;
    const psz_predictor pred = h->pipeline.predictor;
    if (pred != Lorenzo && pred != LorenzoZigZag && pred != Spline) return PSZ_ABORT_NO_SUCH_PREDICTOR;
    if (h->pipeline.codec1 != Huffman) return PSZ_ABORT_NO_SUCH_CODEC;
    const bool zz = pred == LorenzoZigZag;
    const bool spl = pred == Spline;
    if (spl && !d_spl_slots) {  // spline outlier slots: one range per 32x8x8 tile, allocated on first use
      spl_slot_cells = (size_t)sgeom.ntiles * spl_cap;
      CUSZ_AMD_HIP_CHECK(hipMalloc(&d_spl_slots, spl_slot_cells * 8));
      CUSZ_AMD_HIP_CHECK(hipMalloc(&d_spl_cnt, (size_t)sgeom.ntiles * 4));
      CUSZ_AMD_HIP_CHECK(hipMalloc(&d_spl_off, ((size_t)sgeom.ntiles + 1) * 4));
      CUSZ_AMD_HIP_CHECK(hipMalloc(&d_spl_sps, (size_t)sgeom.ntiles * 4));
    }
    const int radius = h->rc.radius;
    const int bklen = 2 * radius;
    if (radius < 1 || bklen > kMaxBklen) return PSZ_AMD_ERR_INVALID_ARG;

    const bool brick = use_brick(pred);
    // chunk length: the caller's, else the tuned one
    if (!brick) {
      const int s = user_sublen ? std::min(8192, ((user_sublen + 255) / 256) * 256) : tuned_sublen;
      if (s != sublen) {
        sublen = s;
        pardeg = (int)((n - 1) / s + 1);
        CUSZ_AMD_HIP_CHECK(alloc_chunk_state());
      }
    }

    mark(0);
    // Rel mode: eb *= (max - min)  (libcusz.cc:287-293; range in double of T extrema)
    if (h->rc.mode == Rel) {
      CUSZ_AMD_HIP_CHECK((hipError_t)launch_extrema<T>(in, n, minmax(), ext_scratch(), stream));
      int fs = fetch(regions({{h_readback() + 512, minmax(), 16}}), 1);
      if (fs) return fs;
      double mm[2];
      std::memcpy(mm, h_readback() + 512, 16);
      h->min_val = mm[0], h->max_val = mm[1];
      h->rc.eb *= (mm[1] - mm[0]);
    }
    const double eb = h->rc.eb;

    // per-call state reset (the reference never resets these: SURVEY.md Appendix B.3)
    if (brick)
      CUSZ_AMD_HIP_CHECK((hipError_t)launch_zero(regions({{d_hist, nullptr, (size_t)(bklen + 1) * 4},
                                                          {d_small, nullptr, kSmallZeroBytes},
                                                          {d_shist, nullptr, ((size_t)kMaxBklen * kSampleBinStride + 16) * 4}}),
                                                 stream));
    else
      CUSZ_AMD_HIP_CHECK((hipError_t)launch_zero(regions({{d_hist, nullptr, (size_t)(bklen + 1) * 4},
                                                          {d_small, nullptr, kSmallZeroBytes},
                                                          {d_status, nullptr, status_words * 8}}),
                                                 stream));
    mark(1);
    last_layout = brick ? PSZ_AMD_LAYOUT_BRICK : PSZ_AMD_LAYOUT_REFERENCE;
    pend.brick = brick, pend.spl = spl, pend.radius = radius, pend.zz = zz;
    pend.anchor_bytes = spl ? sizeof(T) * sgeom.anchor_len : 0;
    if (brick) {
      OutlierSink bol{d_slots, d_brick_cnt, d_spill, spill_cnt(), brick_cap(), spill_cap, nullptr};
      HostPub hp;
      const bool sampled_mode = codebook != PSZ_AMD_CODEBOOK_EXACT;
      BrickSample sample;
      if (sampled_mode && pub_hist && (bl.g.ndim == 3 || bl.g.ndim == 1)) {
        // a single-process compress: pass 1 visits a sample of the bricks first, counts them into
        // d_shist and hands the completed sample to the host, which builds the codebook (the
        // two-queue book of sample + 1) while pass 1 goes on; the encode launches wait behind
        // the device-polled gate as in the exact mode, but the book is ready long before
        sample = brick_sample_plan(bl.g.nbricks, d_shist, d_shist + (size_t)kMaxBklen * kSampleBinStride);
        sample.pub_dst = h_hist(), sample.pub_flag = const_cast<uint32_t*>(flag(2)), sample.pub_epoch = ++epoch;
        sample.bklen = bklen;
        pend.side_book = true;  // (the sample's epoch is pend.hist_epoch)
      }
      if (pub_hist && !pend.side_book)  // (2-D bricks: the full histogram, as in the exact mode)
        hp = HostPub{regions({{h_hist(), d_hist, (size_t)bklen * 4}}), const_cast<uint32_t*>(flag(2)), ++epoch,
                     hist_ticket()};
      pend.hist_epoch = pend.side_book ? sample.pub_epoch : hp.epoch;
      CUSZ_AMD_HIP_CHECK((hipError_t)launch_brick_scan<T>(bl, in, eb, radius, zz, sample, bol, d_hist, d_bhist,
                                                          brick_codes(zz, radius), bklen, stream, hp));
      mark(2);
      pend.active = true;
      return PSZ_SUCCESS;
    }

    const size_t anchor_bytes = spl ? sizeof(T) * sgeom.anchor_len : 0;
    uint64_t* slots = spl ? d_spl_slots : d_slots;
    uint32_t* bcnt = spl ? d_spl_cnt : d_brick_cnt;
    uint32_t* boff = spl ? d_spl_off : d_brick_off;
    const uint32_t nbr = spl ? sgeom.ntiles : geom.nbricks;
    const uint32_t cap = spl ? spl_cap : cap_per_brick;
    OutlierSink ol{slots, bcnt, d_spill, spill_cnt(), cap, spill_cap, spl ? d_spl_sps : nullptr};
    if (spl) {
      SplineArgs<T> sa{in,
                       (uint32_t)len.x,
                       (uint32_t)len.y,
                       (uint32_t)len.z,
                       sgeom.gdx,
                       sgeom.gdy,
                       sgeom.gdz,
                       sgeom.ntiles,
                       (float)(1.0 / eb),
                       (float)(eb * 2.0),
                       radius,
                       bklen,
                       d_codes,
                       reinterpret_cast<T*>(d_archive + 176),
                       ol,
                       d_hist};
      pend.hist_epoch = 0;  // compress_finish publishes the histogram itself
      CUSZ_AMD_HIP_CHECK((hipError_t)launch_spline3_c<T>(sa, stream));
    }
    else {
      // the kernel's last workgroup publishes the histogram to the host (no publish launch) for
      // the host's reference codebook (every mode: measured faster than the device book here)
      HostPub hp;
      if (pub_hist)
        hp = HostPub{regions({{h_hist(), d_hist, (size_t)bklen * 4}}), const_cast<uint32_t*>(flag(2)), ++epoch,
                     hist_ticket()};
      pend.hist_epoch = hp.epoch;
      CUSZ_AMD_HIP_CHECK((hipError_t)launch_lorenzo_c<T>(in, len.x, len.y, len.z, eb, radius, zz, geom, d_codes,
                                                         ol, d_hist, bklen, stream, hp));
    }
    mark(2);
    pend.active = true;
    return PSZ_SUCCESS;
  }

  // Codebook (from d_hist, or from `ext_hist`: a device u32[bklen] the caller reduced across
  // slabs) -> encode -> archive.
  int compress_finish(psz_header* h, const uint32_t* ext_hist, uint8_t** out, size_t* outlen)
  {
    if (!pend.active) return PSZ_AMD_ERR_STATE;
    pend.active = false;
    const int radius = pend.radius, bklen = 2 * radius;
    pend.ext = ext_hist != nullptr;
    if (ext_hist) {
      // bklen counts + the summed overflow word of every slab (psz_amd_compress_scan_*)
      CUSZ_AMD_HIP_CHECK(hipMemcpyAsync(d_hist, ext_hist, (size_t)(bklen + 1) * 4, hipMemcpyDeviceToDevice, stream));
      pend.hist_epoch = 0;  // the scan's published histogram is not the one to encode with
    }
    if (pend.brick) return compress_brick(h, out, outlen, radius);
    const bool spl = pend.spl;
    const size_t anchor_bytes = pend.anchor_bytes;
    uint64_t* slots = spl ? d_spl_slots : d_slots;
    uint32_t* bcnt = spl ? d_spl_cnt : d_brick_cnt;
    uint32_t* boff = spl ? d_spl_off : d_brick_off;
    const uint32_t nbr = spl ? sgeom.ntiles : geom.nbricks;
    const uint32_t cap = spl ? spl_cap : cap_per_brick;
    uint32_t* spill_start = spl ? d_spl_sps : nullptr;

    // codebook: the reference's heap on the host (hf_hl.cc:21-34) when the predictor's last
    // workgroup already published the histogram (Lorenzo, single process: config 1 book stage
    // 9 us against 46 us for the device book), else -- spline, a sharded finish -- on the device
    // from the full histogram unless PSZ_AMD_CODEBOOK_EXACT (no host round trip).  On the host path,
    // as in the brick path, every launch after the book is queued now behind a device-polled
    // gate, and the last kernel publishes the summary: the histogram's trip to the host overlaps
    // nothing, but no launch waits on the host's build.
    const bool host_book = codebook == PSZ_AMD_CODEBOOK_EXACT || pend.hist_epoch != 0;
    uint32_t eh = 0, eg = 0;
    bool gated = false;
    struct GateGuard {  // the gate opens on every path out of here (see compress_brick)
      volatile uint32_t* f;
      uint32_t e;
      bool armed;
      ~GateGuard()
      {
        if (armed) __atomic_store_n(f, e, __ATOMIC_RELEASE);
      }
    } guard{flag(5), 0, false};
    auto build_book = [&]() -> int {
      int fs = wait_flag(2, eh);
      if (!fs) build_codebook(h_hist(), bklen, h_book(), h_revbook());
      if (gated) __atomic_store_n(flag(5), eg, __ATOMIC_RELEASE);  // always open the gate
      guard.armed = false;
      return fs;
    };
    if (host_book) {
      eh = pend.hist_epoch;  // published by the Lorenzo kernel's last workgroup, or now
      if (!eh) {
        eh = ++epoch;
        CUSZ_AMD_HIP_CHECK((hipError_t)launch_publish(hist_regions(bklen), const_cast<uint32_t*>(flag(2)), eh, stream));
      }
      eg = ++gate_epoch;
      gated = gate;
      guard.e = eg, guard.armed = gated;
      if (!gated)
        if (int fs = build_book()) return fs;
    }
    const size_t phf_off = 176 + anchor_bytes;  // anchors: spline only (compressor.inl:160)
    const size_t rvbk = rvbk_bytes(bklen);
    const size_t nbit_rel = 128 + rvbk, entry_rel = nbit_rel + 4 * (size_t)pardeg;
    const size_t bits_rel = entry_rel + 4 * (size_t)pardeg;
    if (!host_book)
      CUSZ_AMD_HIP_CHECK((hipError_t)launch_book_device(d_hist, bklen, 0u, d_book, d_archive + phf_off + 128, stream));
    else {
      const XferRegions up =
          regions({{d_book, h_book(), (size_t)bklen * 4}, {d_archive + phf_off + 128, h_revbook(), rvbk}});
      if (gated)
        CUSZ_AMD_HIP_CHECK((hipError_t)launch_gate_upload(up, const_cast<const uint32_t*>(flag(5)), eg, timeout(), stream));
      else
        CUSZ_AMD_HIP_CHECK((hipError_t)launch_upload(up, stream));
    }
    mark(3);

    HfEncodeArgs ea{d_codes,
                    n,
                    d_book,
                    bklen,
                    sublen,
                    pardeg,
                    reinterpret_cast<uint32_t*>(d_archive + phf_off + nbit_rel),
                    reinterpret_cast<uint32_t*>(d_archive + phf_off + entry_rel),
                    reinterpret_cast<uint32_t*>(d_archive + phf_off + bits_rel),
                    d_status,
                    timeout(),
                    d_enc_temp};
    ea.total_nbit = &info()->total_nbit;  // summed by the encoder's tile-sum pass
    ea.ticket = plan_ticket();            // (the brick plan's ticket: unused on this path)
    CUSZ_AMD_HIP_CHECK((hipError_t)launch_hf_encode(ea, stream));
    mark(4);

    // header templates: static fields from the host, dynamic ones filled on the device (by the
    // finalize workgroup, which knows the totals)
    h->vle_sublen = sublen;
    h->vle_pardeg = pardeg;
    h->len = len;
    h->entry[0] = 0, h->entry[1] = 176, h->entry[2] = (uint32_t)phf_off;
    phf_header ph;
    std::memset(&ph, 0, sizeof(ph));
    ph.bklen = bklen, ph.sublen = sublen, ph.pardeg = pardeg, ph.original_len = n;
    ph.entry[0] = 0, ph.entry[1] = 128, ph.entry[2] = (uint32_t)nbit_rel, ph.entry[3] = (uint32_t)entry_rel;
    ph.entry[4] = (uint32_t)bits_rel;
    FinalizeArgs fa{ea.par_nbit, ea.par_entry, pardeg, bcnt, nbr, cap, spill_cnt(), spill_cap, boff, info(),
                    spill_start};
    fa.nbit_known = true;
    CUSZ_AMD_HIP_CHECK((hipError_t)launch_finalize_scan(fa, stream, h, &ph, d_archive, phf_off, bits_rel));
    OutlierCopyArgs oa{slots, bcnt,      boff,           nbr, cap, d_spill, spill_cnt(), spill_cap,
                       info(), d_archive, phf_off + bits_rel, spill_start};
    // the copy's last workgroup publishes the summary finish_compress reads (no publish launch)
    // when its grid is small; a large grid pays the publish per block, so a publish launch follows
    const HostPub sp{readback_regions(), const_cast<uint32_t*>(flag(3)), ++epoch, summary_ticket()};
    const bool in_copy = nbr <= 4096u;
    CUSZ_AMD_HIP_CHECK((hipError_t)launch_outlier_copy(oa, stream, in_copy ? sp : HostPub{}));
    if (!in_copy)
      CUSZ_AMD_HIP_CHECK((hipError_t)launch_publish(sp.r, sp.flag, sp.epoch, stream));
    summary_epoch = sp.epoch;
    mark(5);
    if (gated)
      if (int fs = build_book()) return fs;
    return finish_compress(h, out, outlen);
  }

  // Fused brick compress (brick.hip): pass 1 (histograms + outliers) -> host codebook ->
  // region reservation -> pass 2 (predict + pack straight into the archive) -> finalize.
  BrickCodes brick_codes(bool zz, int radius) const
  {
    return BrickCodes{d_codes, d_codes8, d_rowmask, zz ? 0u : (uint32_t)std::max(radius - 127, 0)};
  }

  int compress_brick(psz_header* h, uint8_t** out, size_t* outlen, int radius)
  {
    const int bklen = 2 * radius;
    const BrickGeom& g = bl.g;
    const int bsub = g.W, bpar = (int)g.nchunks;
    const uint32_t cap = brick_cap();
    // The histogram goes to the host; the codebook comes back through host-mapped memory.  Every
    // launch after the codebook is queued NOW: the upload kernel polls a host-mapped gate word the
    // host sets once the book is built, so the encode kernels start right after it instead of
    // after the host's launch latency (and without the command processor's stream-wait latency).
    const size_t phf_off = 176;
    const size_t rvbk = rvbk_bytes(bklen);
    const size_t nbit_rel = 128 + rvbk, entry_rel = nbit_rel + 4 * (size_t)bpar;
    const size_t bits_rel = entry_rel + 4 * (size_t)bpar;
    // host book: the reference heap on the full histogram (EXACT; 2-D bricks) or the two-queue
    // book of pass 1's sample + 1 (SAMPLED, published mid-pass); otherwise (a sharded finish) the
    // device book
    const bool sampled = pend.side_book;
    const bool host_book = codebook == PSZ_AMD_CODEBOOK_EXACT || pend.hist_epoch != 0;
    pend.side_book = false;
    uint32_t eh = 0, eg = 0;
    bool gated = false;
    // the gate must open on every path out of here, or the stream (and every later call on
    // it) waits forever: an early error return before build_book() opens it in the destructor
    struct GateGuard {
      volatile uint32_t* f;
      uint32_t e;
      bool armed;
      ~GateGuard()
      {
        if (armed) __atomic_store_n(f, e, __ATOMIC_RELEASE);
      }
    } guard{flag(5), 0, false};
    auto build_book = [&]() -> int {
      int fs = wait_flag(2, eh);
      if (!fs) {
        if (sampled)  // two-queue book of sample + 1 (every code encodable; codebook.cc)
          build_codebook_twoqueue(h_hist(), bklen, 1u, h_book(), h_revbook());
        else
          build_codebook(h_hist(), bklen, h_book(), h_revbook());
      }
      if (gated) __atomic_store_n(flag(5), eg, __ATOMIC_RELEASE);  // always open the gate
      guard.armed = false;
      return fs;
    };
    if (!host_book) {
      // device codebook, no host round trip (a sharded finish: every rank holds the same reduced
      // histogram): built now from the full histogram
      CUSZ_AMD_HIP_CHECK((hipError_t)launch_book_device(d_hist, bklen, 0u, d_book, d_archive + phf_off + 128, stream));
    }
    else {
      eh = pend.hist_epoch;  // published by the scan's last workgroup, or now
      if (!eh) {
        eh = ++epoch;
        CUSZ_AMD_HIP_CHECK((hipError_t)launch_publish(hist_regions(bklen), const_cast<uint32_t*>(flag(2)), eh, stream));
      }
      eg = ++gate_epoch;
      gated = gate;
      guard.e = eg, guard.armed = gated;
      if (!gated)
        if (int fs = build_book()) return fs;
      const XferRegions up =
          regions({{d_book, h_book(), (size_t)bklen * 4}, {d_archive + phf_off + 128, h_revbook(), rvbk}});
      if (gated)
        CUSZ_AMD_HIP_CHECK((hipError_t)launch_gate_upload(up, const_cast<const uint32_t*>(flag(5)), eg, timeout(), stream));
      else
        CUSZ_AMD_HIP_CHECK((hipError_t)launch_upload(up, stream));
    }
    mark(3);

    uint32_t* par_nbit = reinterpret_cast<uint32_t*>(d_archive + phf_off + nbit_rel);
    uint32_t* par_entry = reinterpret_cast<uint32_t*>(d_archive + phf_off + entry_rel);
    uint32_t* bits = reinterpret_cast<uint32_t*>(d_archive + phf_off + bits_rel);

    // header templates: static fields from the host, sizes filled by the plan kernel
    h->vle_sublen = bsub;
    h->vle_pardeg = bpar;
    h->len = len;
    h->entry[0] = 0, h->entry[1] = 176, h->entry[2] = (uint32_t)phf_off;
    phf_header ph;
    std::memset(&ph, 0, sizeof(ph));
    ph.bklen = bklen, ph.sublen = bsub, ph.pardeg = bpar, ph.original_len = n;
    ph.entry[0] = 0, ph.entry[1] = 128, ph.entry[2] = (uint32_t)nbit_rel, ph.entry[3] = (uint32_t)entry_rel;
    ph.entry[4] = (uint32_t)bits_rel;

    const uint32_t nblk = brick_plan_blocks(g.nbricks);
    BrickPlanArgs pa{d_bhist, bklen, brick_hist_stride(bklen), d_book, g.nbricks, brick_units(g.nbricks), g.nbx, g.nby, bl.ly, bl.lz,
                     d_brick_cnt, cap, d_slots, d_spill, spill_cnt(), spill_cap, nblk, d_ub, d_bbase, d_brick_off,
                     d_plan, d_plan + nblk + 1, info(), d_archive, phf_off, bits_rel};
    pa.nd = g.ndim == 3 ? 3u : 1u, pa.nchunks = g.nchunks, pa.n = g.n;  // 1-D and 2-D: linear bricks
    pa.ticket = plan_ticket();
    CUSZ_AMD_HIP_CHECK((hipError_t)launch_brick_plan(bl, pa, h, &ph, stream));
    // the pack's last workgroup publishes the summary finish_compress reads (no publish launch)
    const HostPub sp{readback_regions(), const_cast<uint32_t*>(flag(3)), ++epoch, summary_ticket()};
    CUSZ_AMD_HIP_CHECK((hipError_t)launch_brick_pack(bl, brick_codes(pend.zz, radius), d_book, bklen, pa, par_nbit, par_entry, bits,
                                                     pack_reverse, timeout(), stream, sp));
    summary_epoch = sp.epoch;
    mark(4);
    if (gated)
      if (int fs = build_book()) return fs;
    mark(5);
    return finish_compress(h, out, outlen);
  }

  // Single-pass mode (PSZ_AMD_CODEBOOK_STREAM, 3-D bricks): the sample kernel hands the histogram
  // of every 16th 32 x 8 x 8 unit to the host, which builds the two-queue book of sample + 1 while
  // the streaming pass predicts its first bricks; that pass takes the book behind a device-polled
  // gate, sizes each brick (one workgroup per brick), takes its offset by a look-back and writes
  // its rows straight to the archive; a finish kernel writes the outlier segment and the headers.
  // Codes, outliers and the reconstruction equal the exact mode's; the bitstream does not.
  template <typename T>
  int compress_sampled(psz_header* h, const T* in, uint8_t** out, size_t* outlen)
  {
    pend.active = false;
    pend.ext = false;  // no caller's overflow word in this mode (finish_compress reads it when set)
    pend.spl = false, pend.brick = true;
    if (h->pipeline.codec1 != Huffman) return PSZ_ABORT_NO_SUCH_CODEC;
    const bool zz = h->pipeline.predictor == LorenzoZigZag;
    const int radius = h->rc.radius, bklen = 2 * radius;
    if (radius < 1 || bklen > kMaxBklen) return PSZ_AMD_ERR_INVALID_ARG;
    const BrickGeom& g = bl.g;
    mark(0);
    if (h->rc.mode == Rel) {  // libcusz.cc:287-293
      CUSZ_AMD_HIP_CHECK((hipError_t)launch_extrema<T>(in, n, minmax(), ext_scratch(), stream));
      int fs = fetch(regions({{h_readback() + 512, minmax(), 16}}), 1);
      if (fs) return fs;
      double mm[2];
      std::memcpy(mm, h_readback() + 512, 16);
      h->min_val = mm[0], h->max_val = mm[1];
      h->rc.eb *= (mm[1] - mm[0]);
    }
    const double eb = h->rc.eb;
    // the look-back status words (one per brick), then the outlier count and destination of each
    // (brick, y-step) slot, live in the per-brick histogram area (unused in this mode: 2 KB a brick)
    unsigned long long* status = reinterpret_cast<unsigned long long*>(d_bhist);
    uint32_t* slot_cnt = reinterpret_cast<uint32_t*>(status + g.nbricks);
    uint32_t* slot_dst = slot_cnt + (size_t)g.nbricks * kStreamSlots;
    CUSZ_AMD_HIP_CHECK((hipError_t)launch_zero(regions({{d_shist, nullptr, (size_t)kMaxBklen * kSampleBinStride * 4},
                                                        {d_small, nullptr, kSmallZeroBytes},
                                                        {status, nullptr, (size_t)g.nbricks * 8}}),
                                               stream));
    mark(1);
    last_layout = PSZ_AMD_LAYOUT_BRICK;
    const size_t phf_off = 176;
    const size_t rvbk = rvbk_bytes(bklen);
    const int bsub = g.W, bpar = (int)g.nchunks;
    const size_t nbit_rel = 128 + rvbk, entry_rel = nbit_rel + 4 * (size_t)bpar;
    const size_t bits_rel = entry_rel + 4 * (size_t)bpar;
    // the sample histogram; its last workgroup publishes it to the host (flag 2)
    const uint32_t eh = ++epoch;
    CUSZ_AMD_HIP_CHECK((hipError_t)launch_brick_sample<T>(bl, in, eb, radius, zz, d_shist, bklen, hist_ticket(), h_hist(),
                                                          const_cast<uint32_t*>(flag(2)), eh, stream));
    mark(2);
    // the host's two-queue book of sample + 1 opens the gate the streaming pass polls; it must
    // open on every path out of here, or the stream (and every later call on it) waits forever
    const uint32_t eg = ++gate_epoch;
    struct GateGuard {
      volatile uint32_t* f;
      uint32_t e;
      bool armed;
      ~GateGuard()
      {
        if (armed) __atomic_store_n(f, e, __ATOMIC_RELEASE);
      }
    } guard{flag(5), eg, true};
    auto build_book = [&]() -> int {
      int fs = wait_flag(2, eh);
      if (!fs) build_codebook_twoqueue(h_hist(), bklen, 1u, h_book(), h_revbook());
      __atomic_store_n(flag(5), eg, __ATOMIC_RELEASE);
      guard.armed = false;
      return fs;
    };
    if (!gate)  // (diagnostic switch: the book before the launch)
      if (int fs = build_book()) return fs;
    mark(3);
    h->vle_sublen = bsub;
    h->vle_pardeg = bpar;
    h->len = len;
    h->entry[0] = 0, h->entry[1] = 176, h->entry[2] = (uint32_t)phf_off;
    phf_header ph;
    std::memset(&ph, 0, sizeof(ph));
    ph.bklen = bklen, ph.sublen = bsub, ph.pardeg = bpar, ph.original_len = n;
    ph.entry[0] = 0, ph.entry[1] = 128, ph.entry[2] = (uint32_t)nbit_rel, ph.entry[3] = (uint32_t)entry_rel;
    ph.entry[4] = (uint32_t)bits_rel;
    const size_t chunks = std::max((size_t)pardeg, (size_t)g.nchunks);
    BrickSingle sg{OutlierSink{d_slots, slot_cnt, d_spill, spill_cnt(), brick_cap() / kStreamSlots, spill_cap, nullptr},
                   d_book,
                   bklen,
                   reinterpret_cast<uint32_t*>(d_archive + phf_off + nbit_rel),
                   reinterpret_cast<uint32_t*>(d_archive + phf_off + entry_rel),
                   reinterpret_cast<uint32_t*>(d_archive + phf_off + bits_rel),
                   (uint32_t)std::min<size_t>(bitstream_cells_cap() + chunks, 0xFFFFFFFFu),
                   status,
                   &info()->ticket,
                   slot_dst,
                   info(),
                   timeout(),
                   d_archive,
                   phf_off,
                   bits_rel,
                   const_cast<const uint32_t*>(flag(5)),
                   eg,
                   h_book(),
                   reinterpret_cast<const uint32_t*>(h_revbook()),
                   reinterpret_cast<uint32_t*>(d_archive + phf_off + 128),
                   (int)(rvbk / 4),
                   book_flag()};
    const HostPub sp{readback_regions(), const_cast<uint32_t*>(flag(3)), ++epoch, summary_ticket()};
    CUSZ_AMD_HIP_CHECK((hipError_t)launch_brick_stream<T>(bl, in, eb, radius, zz, sg, h, &ph, stream, sp));
    summary_epoch = sp.epoch;
    mark(4);
    mark(5);
    if (guard.armed)
      if (int fs = build_book()) return fs;
    return finish_compress(h, out, outlen);
  }

  // read back the device-written header + summary (one flag wait), report status
  // the histogram for the host codebook, and with a caller's reduced histogram its overflow word
  XferRegions hist_regions(int bklen)
  {
    if (pend.ext) return regions({{h_hist(), d_hist, (size_t)bklen * 4}, {h_readback() + 448, d_hist + bklen, 4}});
    return regions({{h_hist(), d_hist, (size_t)bklen * 4}});
  }
  uint32_t global_excess() const { return pend.ext ? *reinterpret_cast<const uint32_t*>(h_readback() + 448) : 0u; }

  XferRegions readback_regions()
  {
    // a sharded finish also reads back the summed overflow word (the device-book path sends no
    // histogram to the host)
    if (pend.ext)
      return regions({{h_readback(), d_archive, 176},
                      {h_readback() + 256, info(), sizeof(CompressInfo)},
                      {h_readback() + 384, timeout(), 4},
                      {h_readback() + 448, d_hist + 2 * pend.radius, 4}});
    return regions({{h_readback(), d_archive, 176},
                    {h_readback() + 256, info(), sizeof(CompressInfo)},
                    {h_readback() + 384, timeout(), 4}});
  }

  int finish_compress(psz_header* h, uint8_t** out, size_t* outlen)
  {
    const uint32_t se = summary_epoch;
    summary_epoch = 0;
    int fs = se ? wait_flag(3, se) : fetch(readback_regions(), 3);
    if (fs) return fs;
    if (timing) CUSZ_AMD_HIP_CHECK(hipEventSynchronize(ev[5]));
    CompressInfo ci;
    std::memcpy(&ci, h_readback() + 256, sizeof(ci));
    unsigned int tmo;
    std::memcpy(&tmo, h_readback() + 384, 4);
    std::memcpy(h, h_readback(), 176);
    splen = (size_t)ci.splen;
    if (timing) {
      stage_ms[PSZ_AMD_T_EXTREMA] = span(0, 1);
      stage_ms[PSZ_AMD_T_PREDICT] = span(1, 2);
      stage_ms[PSZ_AMD_T_BOOK] = span(2, 3);
      stage_ms[PSZ_AMD_T_ENCODE] = span(3, 4);
      stage_ms[PSZ_AMD_T_FINALIZE] = span(4, 5);
      stage_ms[PSZ_AMD_T_COMPRESS] = span(0, 5);
    }
    if (tmo) {
      std::fprintf(stderr, "[cusz_amd] encoder reservation/look-back check failed\n");
      return PSZ_AMD_ERR_ENCODER;
    }
    if (ci.spilled && !pend.spl) {
      // bricks spilled past their slots: grow the slots to the largest brick's count so that the
      // repeat writes every cell in its brick's slot (deterministic order, fused decoders' ranked
      // reads); compress() then runs once more, a scan/finish caller gets the warning and repeats
      const int g = grow_slots(ci.max_brick_cnt);
      if (g < 0) return PSZ_AMD_ERR_DEVICE;
      if (g > 0) return PSZ_WARN_OUTLIER_TOO_MANY;
    }
    if (ci.outlier_lost) {
      // the spill list was too small for this field's outliers (every cell was counted): grow it
      // (and the archive) to hold them all; compress() then runs once more, a scan/finish caller
      // gets the warning and repeats scan and finish
      const int g = grow_spill((uint64_t)spill_cap + ci.outlier_lost);
      if (g < 0) return PSZ_AMD_ERR_DEVICE;
      return PSZ_WARN_OUTLIER_TOO_MANY;
    }
    // a sharded finish: another slab overflowed (the summed overflow word), so every rank sees
    // the warning and repeats the step together
    const uint32_t gx = global_excess();
    pend.ext = false;  // consumed: a later call never reads this finish's overflow word
    if (gx) return PSZ_WARN_OUTLIER_TOO_MANY;
    *out = d_archive;
    *outlen = h->entry[PSZHEADER_ENC_PASS2_END];
    return PSZ_SUCCESS;
  }

  int decode_codes(const psz_header* h, const uint8_t* in)
  {
    // the decoders write d_codes, which a pending compress_finish would pack (as decompress)
    pend.active = false;
    const int bklen = 2 * h->rc.radius;
    const size_t phf_off = h->entry[PSZHEADER_ENCODED];
    const size_t rvbk = rvbk_bytes(bklen);
    const int pd = h->vle_pardeg, sl = h->vle_sublen;
    const uint8_t* phf = in + phf_off;
    if (sl % 64 == 0 && sl <= 8192 && decoder == 0 && pd > 0 && bklen <= kMaxBklen) {  // the fused decoders' chunk loop
      const size_t bits_off = phf_off + 128 + rvbk + 8 * (size_t)pd;
      const size_t total = h->entry[PSZHEADER_ENC_PASS2_END];
      const size_t bs_words = total > bits_off ? (total - bits_off) / 4 : 0;
      CUSZ_AMD_HIP_CHECK((hipError_t)launch_chunk_decode(
          bl, reinterpret_cast<const uint32_t*>(phf + 128 + rvbk + 8 * (size_t)pd), bs_words, phf + 128, bklen,
          reinterpret_cast<const uint32_t*>(phf + 128 + rvbk), reinterpret_cast<const uint32_t*>(phf + 128 + rvbk + 4 * (size_t)pd),
          d_codes, n, (uint32_t)pd, (uint32_t)sl, stream));
      return PSZ_SUCCESS;
    }
    HfDecodeArgs da{reinterpret_cast<const uint32_t*>(phf + 128 + rvbk + 8 * (size_t)pd),
                    phf + 128,
                    bklen,
                    reinterpret_cast<const uint32_t*>(phf + 128 + rvbk),
                    reinterpret_cast<const uint32_t*>(phf + 128 + rvbk + 4 * (size_t)pd),
                    sl,
                    pd,
                    n,
                    d_codes,
                    dec_lut(),
                    0,
                    decoder};
    // average chunk size from the segment length (sizes the decoder's LDS staging)
    const size_t seg = h->entry[PSZHEADER_ENCODED + 1] - h->entry[PSZHEADER_ENCODED];
    const size_t fixed = 128 + rvbk + 8 * (size_t)pd;
    if (pd > 0 && seg > fixed) da.avg_cells = (seg - fixed) / 4 / (size_t)pd;
    CUSZ_AMD_HIP_CHECK((hipError_t)launch_hf_decode(da, stream));
    return PSZ_SUCCESS;
  }

  template <typename T>
  int decompress(const psz_header* h, const uint8_t* in, T* out)
  {
    // the decoders overwrite the code buffer a pending compress_finish would pack: a scan ->
    // decompress -> finish sequence must fail cleanly instead of writing a corrupt archive
    pend.active = false;
    const psz_predictor pred = h->pipeline.predictor;
    if (pred != Lorenzo && pred != LorenzoZigZag && pred != Spline) return PSZ_ABORT_NO_SUCH_PREDICTOR;
    const bool zz = pred == LorenzoZigZag;
    if (h->len.x != len.x || h->len.y != len.y || h->len.z != len.z) return PSZ_ABORT_UNSUPPORTED_DIMENSION;
    if (pred == Spline) return decompress_spline<T>(h, in, out);
    mark(6);
    // fused decode + reconstruct: 3-D and 1-D (2-D linear-brick archives decode chunk by chunk)
    const bool brickdec = bl.g.ok && bl.g.ndim != 2 && decoder == 0 && h->vle_sublen == bl.g.W &&
                          2 * h->rc.radius <= kMaxBklen;
    const uint32_t* cells = reinterpret_cast<const uint32_t*>(in + h->entry[PSZHEADER_SPFMT]);
    X1dOutliers ox;  // 1-D: the reconstruction reads sorted cells directly (no scatter pass)
    if (geom.ndim == 1 && d_x1d && !zz && !brickdec && h->splen) {
      const uint32_t nb = geom.nbricks;
      CUSZ_AMD_HIP_CHECK((hipError_t)launch_x1d_bounds(cells, h->splen, n, nb, d_x1d, d_x1d + nb + 1,
                                                       next_cell_epoch(), stream));
      ox = X1dOutliers{cells, (size_t)h->splen, d_x1d, d_x1d + nb + 1, cell_epoch};
    }
    // fused brick path: the decoder ranks each row's zero codes against the brick's cells when
    // they are grouped and sorted; only otherwise does the scatter below run (only_if = unsorted)
    BrickOutliers bo;
    if (brickdec && !zz && h->splen) {
      // cells per brick (3-D) or per chunk (1-D)
      const uint32_t nb = bl.g.ndim == 1 ? bl.g.nchunks : bl.g.nbricks;
      if (bl.g.ndim == 1)
        CUSZ_AMD_HIP_CHECK((hipError_t)launch_x1d_bounds(cells, h->splen, n, nb, d_x1d, d_x1d + nb + 1,
                                                         next_cell_epoch(), stream, 8));
      else
        CUSZ_AMD_HIP_CHECK((hipError_t)launch_brick_cell_bounds(bl, cells, h->splen, d_x1d, d_x1d + nb + 1,
                                                                next_cell_epoch(), stream));
      bo = BrickOutliers{cells, (size_t)h->splen, d_x1d, d_x1d + nb + 1, cell_epoch};
      ox.unsorted = bo.unsorted;
      ox.epoch = cell_epoch;
    }
    if (zz) CUSZ_AMD_HIP_CHECK(hipMemsetAsync(out, 0, n * sizeof(T), stream));
    CUSZ_AMD_HIP_CHECK((hipError_t)launch_scatter<T>(cells, h->splen, out, n, stream, ox.unsorted, ox.epoch));
    mark(7);
    if (brickdec) return decompress_brick<T>(h, in, out, zz, bo);
    int s = decode_codes(h, in);
    if (s) return s;
    mark(8);
    CUSZ_AMD_HIP_CHECK((hipError_t)launch_lorenzo_x<T>(d_codes, out, len.x, len.y, len.z, h->rc.eb, h->rc.radius,
                                                       zz, geom, stream, ox.cells ? &ox : nullptr));
    mark(9);
    return PSZ_SUCCESS;
  }

  // fused decode + reconstruct (brick.hip): any archive whose chunk length is the brick width
  template <typename T>
  int decompress_brick(const psz_header* h, const uint8_t* in, T* out, bool zz, const BrickOutliers& bo)
  {
    const int bklen = 2 * h->rc.radius;
    const size_t phf_off = h->entry[PSZHEADER_ENCODED];
    const size_t rvbk = rvbk_bytes(bklen);
    const int pd = h->vle_pardeg;
    const uint8_t* phf = in + phf_off;
    // words from the bitstream start to the end of the archive (range of the decoder's loads)
    const size_t bits_off = phf_off + 128 + rvbk + 8 * (size_t)pd;
    const size_t total = h->entry[PSZHEADER_ENC_PASS2_END];
    const size_t bs_words = total > bits_off ? (total - bits_off) / 4 : 0;
    CUSZ_AMD_HIP_CHECK((hipError_t)launch_brick_decode<T>(
        bl, reinterpret_cast<const uint32_t*>(phf + 128 + rvbk + 8 * (size_t)pd), bs_words, phf + 128, bklen,
        reinterpret_cast<const uint32_t*>(phf + 128 + rvbk), reinterpret_cast<const uint32_t*>(phf + 128 + rvbk + 4 * (size_t)pd),
        out, h->rc.eb, h->rc.radius, zz, bo, stream));
    mark(8);
    mark(9);
    return PSZ_SUCCESS;
  }

  // decode -> (outlier buckets) -> spline reconstruct; the archive's outlier cells hold codes
  template <typename T>
  int decompress_spline(const psz_header* h, const uint8_t* in, T* out)
  {
    mark(6);
    const size_t words = spline_x_scratch_words(sgeom.ntiles, h->splen);
    if (words > spl_x_words) {
      if (d_spl_x) (void)hipFree(d_spl_x), d_spl_x = nullptr;
      CUSZ_AMD_HIP_CHECK(hipMalloc(&d_spl_x, words * 4));
      spl_x_words = words;
    }
    mark(7);
    int s = decode_codes(h, in);
    if (s) return s;
    mark(8);
    const double eb = h->rc.eb;
    SplineXArgs<T> xa{d_codes,
                      reinterpret_cast<const T*>(in + h->entry[PSZHEADER_ANCHOR]),
                      out,
                      (uint32_t)len.x,
                      (uint32_t)len.y,
                      (uint32_t)len.z,
                      sgeom.gdx,
                      sgeom.gdy,
                      sgeom.gdz,
                      sgeom.ntiles,
                      (float)(1.0 / eb),
                      (float)(eb * 2.0),
                      (int)h->rc.radius};
    CUSZ_AMD_HIP_CHECK((hipError_t)launch_spline3_x<T>(
        xa, reinterpret_cast<const uint32_t*>(in + h->entry[PSZHEADER_SPFMT]), h->splen, d_spl_x, stream));
    mark(9);
    return PSZ_SUCCESS;
  }

  void collect_decompress_times()
  {
    if (!timing) return;
    (void)hipEventSynchronize(ev[9]);
    stage_ms[PSZ_AMD_T_SCATTER] = span(6, 7);
    stage_ms[PSZ_AMD_T_DECODE] = span(7, 8);
    stage_ms[PSZ_AMD_T_RECON] = span(8, 9);
    stage_ms[PSZ_AMD_T_DECOMPRESS] = span(6, 9);
  }
};

static Pipeline* P(psz_resource* m) { return m ? reinterpret_cast<Pipeline*>(m->buf) : nullptr; }

}  // namespace cusz_amd

using cusz_amd::Pipeline;

// =========================================================================================
// resource-manager API (cusz_rev1.h)
// =========================================================================================

static thread_local int g_create_status = PSZ_SUCCESS;  // psz_amd_last_create_status

static psz_resource* make_resource(psz_header* hdr, void* stream)
{
  g_create_status = PSZ_AMD_ERR_DEVICE;  // allocation failures below
  auto* m = new (std::nothrow) psz_resource;
  if (!m) return nullptr;
  std::memset(m, 0, sizeof(*m));
  m->header = hdr;
  m->len_linear = hdr->len.x * hdr->len.y * hdr->len.z;
  m->stream = stream;
  m->device = AMDGPU;
  m->dict_size = (uint16_t)(hdr->rc.radius * 2);
  auto* p = new (std::nothrow) Pipeline;
  if (!p) {
    delete m;
    return nullptr;
  }
  int st = p->init(hdr->dtype, hdr->len, stream);
  g_create_status = st;
  m->buf = p;
  m->ndim = p->ndim;
  m->last_error = (psz_error_status)st;
  if (st != PSZ_SUCCESS) {
    delete p;
    delete hdr;
    delete m;
    return nullptr;
  }
  return m;
}

extern "C" {

psz_resource* psz_create_resource_manager(psz_dtype dtype, psz_len len, psz_pipeline pipeline, void* stream)
{
  g_create_status = PSZ_ABORT_UNSUPPORTED_TYPE;
  if (dtype != F4 && dtype != F8) return nullptr;
  g_create_status = PSZ_AMD_ERR_DEVICE;
  auto* h = new (std::nothrow) psz_header;
  if (!h) return nullptr;
  std::memset(h, 0, sizeof(*h));
  h->dtype = dtype;
  h->pipeline = pipeline;
  h->len = len;
  h->rc.radius = DEFAULT_RADIUS;
  h->intp_param = make_default_params();
  auto* m = make_resource(h, stream);
  if (m) phf_coarse_tune(m->len_linear, &h->vle_sublen, &h->vle_pardeg);
  return m;
}

psz_resource* psz_create_resource_manager_from_header(psz_header* header, void* stream)
{
  g_create_status = !header ? PSZ_AMD_ERR_INVALID_ARG : PSZ_ABORT_UNSUPPORTED_TYPE;
  if (!header || (header->dtype != F4 && header->dtype != F8)) return nullptr;
  g_create_status = PSZ_AMD_ERR_DEVICE;
  auto* h = new (std::nothrow) psz_header;
  if (!h) return nullptr;
  std::memcpy(h, header, sizeof(psz_header));
  return make_resource(h, stream);
}

void psz_modify_resource_manager_from_header(psz_resource* m, psz_header* header)
{
  if (!m || !header) return;
  std::memcpy(m->header, header, sizeof(psz_header));
  m->dict_size = (uint16_t)(m->header->rc.radius * 2);
  m->len_linear = header->len.x * header->len.y * header->len.z;
}

int psz_release_resource(psz_resource* m)
{
  if (!m) return PSZ_SUCCESS;
  delete cusz_amd::P(m);
  delete m->cli;
  delete m->header;
  delete m;
  return PSZ_SUCCESS;
}

}  // extern "C"

template <typename T>
static int compress_impl(psz_resource* m, psz_rc2 rc, T* in, psz_header* out_h, uint8_t** out, size_t* outlen)
{
  if (!m || !in || !out || !outlen) return PSZ_AMD_ERR_INVALID_ARG;
  Pipeline* p = cusz_amd::P(m);
  if ((sizeof(T) == 4) != (m->header->dtype == F4)) return PSZ_ABORT_UNSUPPORTED_TYPE;
  int status = PSZ_SUCCESS;
  if (rc.radius > 512) rc.radius = 512, status = PSZ_WARN_RADIUS_TOO_LARGE;  // libcusz.cc:281-285
  m->header->rc = rc;
  m->header->user_input_eb = rc.eb;
  // the value range is this call's (Rel mode) or none: the reference leaves the previous call's
  // range in the header (libcusz.cc:287-293 writes it only in Rel mode), so an Abs archive's
  // bytes would depend on the manager's history (per-call state reset)
  m->header->min_val = m->header->max_val = 0;
  m->dict_size = (uint16_t)(rc.radius * 2);
  CUSZ_AMD_HIP_CHECK(hipSetDevice(p->device));  // the creation device (B.7; several GPUs per process)
  int s = p->compress<T>(m->header, in, out, outlen);
  if (out_h) *out_h = *m->header;
  return s != PSZ_SUCCESS ? s : status;
}

template <typename T>
static int scan_impl(psz_resource* m, psz_rc2 rc, T* in)
{
  if (!m || !in) return PSZ_AMD_ERR_INVALID_ARG;
  Pipeline* p = cusz_amd::P(m);
  if ((sizeof(T) == 4) != (m->header->dtype == F4)) return PSZ_ABORT_UNSUPPORTED_TYPE;
  int status = PSZ_SUCCESS;
  if (rc.radius > 512) rc.radius = 512, status = PSZ_WARN_RADIUS_TOO_LARGE;  // libcusz.cc:281-285
  m->header->rc = rc;
  m->header->user_input_eb = rc.eb;
  m->header->min_val = m->header->max_val = 0;  // as compress_impl
  m->dict_size = (uint16_t)(rc.radius * 2);
  CUSZ_AMD_HIP_CHECK(hipSetDevice(p->device));
  const int s = p->compress_scan<T>(m->header, in);
  return s != PSZ_SUCCESS ? s : status;
}

// copy the slab histogram (device) to the caller's device buffer, on the manager's stream
static int export_hist(psz_resource* m, uint32_t* d_out, int status)
{
  Pipeline* p = cusz_amd::P(m);
  if (!d_out) return PSZ_AMD_ERR_INVALID_ARG;
  const int bklen = 2 * m->header->rc.radius;
  CUSZ_AMD_HIP_CHECK(hipMemcpyAsync(d_out, p->d_hist, sizeof(uint32_t) * bklen, hipMemcpyDeviceToDevice, p->stream));
  // word bklen: this slab's spilled outlier cells -- past its bricks' slots (Lorenzo: every rank
  // then repeats with grown slots, deterministic archives) or past its spill list (spline) --
  // summed with the histograms
  const uint32_t free_spill = p->pend.spl ? p->spill_cap : 0u;
  CUSZ_AMD_HIP_CHECK((hipError_t)cusz_amd::launch_excess(p->spill_cnt(), free_spill, d_out + bklen, p->stream));
  return status;
}

extern "C" {

int psz_compress_float(psz_resource* m, psz_rc2 rc, float* in, psz_header* out_h, uint8_t** out, size_t* outlen)
{
  return compress_impl<float>(m, rc, in, out_h, out, outlen);
}

int psz_compress_double(psz_resource* m, psz_rc2 rc, double* in, psz_header* out_h, uint8_t** out,
                        size_t* outlen)
{
  return compress_impl<double>(m, rc, in, out_h, out, outlen);
}

int psz_compress_analyize_float(psz_resource* m, psz_rc2 rc, float* in, u4* exported_h_hist)
{
  // compressor.inl:305-337: predict + histogram only, the histogram exported to the host
  if (!exported_h_hist) return PSZ_AMD_ERR_INVALID_ARG;
  const int s = scan_impl<float>(m, rc, in);
  if (s != PSZ_SUCCESS && s != PSZ_WARN_RADIUS_TOO_LARGE) return s;
  Pipeline* p = cusz_amd::P(m);
  const size_t bytes = sizeof(u4) * 2 * m->header->rc.radius;
  const int fs = p->fetch(Pipeline::regions({{p->h_hist(), p->d_hist, bytes}}), 2);
  p->pend.active = false;
  if (fs) return fs;
  std::memcpy(exported_h_hist, p->h_hist(), bytes);
  return s;
}

int psz_amd_compress_scan_float(psz_resource* m, psz_rc2 rc, float* in, uint32_t* d_hist_out)
{
  const int s = scan_impl<float>(m, rc, in);
  return (s == PSZ_SUCCESS || s == PSZ_WARN_RADIUS_TOO_LARGE) ? export_hist(m, d_hist_out, s) : s;
}

int psz_amd_compress_scan_double(psz_resource* m, psz_rc2 rc, double* in, uint32_t* d_hist_out)
{
  const int s = scan_impl<double>(m, rc, in);
  return (s == PSZ_SUCCESS || s == PSZ_WARN_RADIUS_TOO_LARGE) ? export_hist(m, d_hist_out, s) : s;
}

int psz_amd_value_range(psz_resource* m, const void* in, size_t len, double* d_minmax)
{
  Pipeline* p = cusz_amd::P(m);
  if (!p || !in || !d_minmax) return PSZ_AMD_ERR_INVALID_ARG;
  if (len == 0) len = p->n;
  CUSZ_AMD_HIP_CHECK(hipSetDevice(p->device));
  if (m->header->dtype == F4)
    CUSZ_AMD_HIP_CHECK((hipError_t)cusz_amd::launch_extrema<float>(static_cast<const float*>(in), len, d_minmax,
                                                                   p->ext_scratch(), p->stream));
  else
    CUSZ_AMD_HIP_CHECK((hipError_t)cusz_amd::launch_extrema<double>(static_cast<const double*>(in), len, d_minmax,
                                                                    p->ext_scratch(), p->stream));
  return PSZ_SUCCESS;
}

int psz_amd_compress_finish(psz_resource* m, const uint32_t* d_hist, psz_header* out_h, uint8_t** out,
                            size_t* outlen)
{
  Pipeline* p = cusz_amd::P(m);
  if (!p || !out || !outlen) return PSZ_AMD_ERR_INVALID_ARG;
  CUSZ_AMD_HIP_CHECK(hipSetDevice(p->device));
  const int s = p->compress_finish(m->header, d_hist, out, outlen);
  if (out_h) *out_h = *m->header;
  return s;
}

}  // extern "C"

template <typename T>
static int decompress_impl(psz_resource* m, uint8_t* in, size_t in_len, T* out)
{
  if (!m || !in || !out) return PSZ_AMD_ERR_INVALID_ARG;
  Pipeline* p = cusz_amd::P(m);
  // the header's segment table must be ordered and fit the archive the caller passed
  const uint32_t* e = m->header->entry;
  for (int k = 1; k <= PSZHEADER_ENC_PASS2_END; k++)
    if (e[k] < e[k - 1]) return PSZ_AMD_ERR_BAD_ARCHIVE;
  if (in_len && e[PSZHEADER_ENC_PASS2_END] > in_len) return PSZ_AMD_ERR_BAD_ARCHIVE;
  if ((size_t)e[PSZHEADER_ENC_PASS1_END] - e[PSZHEADER_SPFMT] != 8 * m->header->splen) return PSZ_AMD_ERR_BAD_ARCHIVE;
  if ((sizeof(T) == 4) != (m->header->dtype == F4)) return PSZ_ABORT_UNSUPPORTED_TYPE;
  CUSZ_AMD_HIP_CHECK(hipSetDevice(p->device));
  int s = p->decompress<T>(m->header, in, out);
  if (s == PSZ_SUCCESS && p->timing) p->collect_decompress_times();
  return s;
}

extern "C" {

int psz_decompress_float(psz_resource* m, uint8_t* in, size_t const in_len, float* out)
{
  return decompress_impl<float>(m, in, in_len, out);
}

int psz_decompress_double(psz_resource* m, uint8_t* in, size_t const in_len, double* out)
{
  return decompress_impl<double>(m, in, in_len, out);
}

// =========================================================================================
// extensions (cusz_amd.h)
// =========================================================================================

int psz_amd_get_internals(psz_resource* m, psz_amd_internals* o)
{
  Pipeline* p = cusz_amd::P(m);
  if (!p || !o) return PSZ_AMD_ERR_INVALID_ARG;
  o->d_quant_codes = p->d_codes;
  o->d_hist = p->d_hist;
  o->d_book = p->d_book;
  o->len = p->n;
  o->bklen = 2 * m->header->rc.radius;
  o->sublen = p->sublen;
  o->pardeg = p->pardeg;
  o->ndim = p->ndim;
  o->splen = p->splen;
  o->archive_capacity = p->archive_cap;
  o->layout = p->last_layout;
  o->brick_width = p->bl.g.ok ? p->bl.g.W : 0;
  return PSZ_SUCCESS;
}

int psz_amd_enable_timing(psz_resource* m, int on)
{
  Pipeline* p = cusz_amd::P(m);
  if (!p) return PSZ_AMD_ERR_INVALID_ARG;
  p->timing = on != 0;
  return PSZ_SUCCESS;
}

int psz_amd_stage_times(psz_resource* m, float* ms, int n)
{
  Pipeline* p = cusz_amd::P(m);
  if (!p || !ms) return PSZ_AMD_ERR_INVALID_ARG;
  for (int i = 0; i < n && i < PSZ_AMD_T_COUNT; i++) ms[i] = p->stage_ms[i];
  return PSZ_SUCCESS;
}

int psz_amd_set_sublen(psz_resource* m, int sublen)
{
  Pipeline* p = cusz_amd::P(m);
  if (!p || sublen < 0) return PSZ_AMD_ERR_INVALID_ARG;
  p->user_sublen = sublen;
  if (sublen == 0) {
    cusz_amd::tune_chunking(p->n, p->device, &p->sublen, &p->pardeg);
    if (p->alloc_chunk_state() != hipSuccess) return PSZ_AMD_ERR_DEVICE;
  }
  return PSZ_SUCCESS;
}

int psz_amd_set_decoder(psz_resource* m, int kind)
{
  Pipeline* p = cusz_amd::P(m);
  if (!p || kind < PSZ_AMD_DECODER_AUTO || kind > PSZ_AMD_DECODER_WAVE) return PSZ_AMD_ERR_INVALID_ARG;
  p->decoder = kind;
  return PSZ_SUCCESS;
}

int psz_amd_set_codebook(psz_resource* m, int mode)
{
  Pipeline* p = cusz_amd::P(m);
  if (!p || (mode != PSZ_AMD_CODEBOOK_EXACT && mode != PSZ_AMD_CODEBOOK_SAMPLED && mode != PSZ_AMD_CODEBOOK_STREAM))
    return PSZ_AMD_ERR_INVALID_ARG;
  p->codebook = mode;
  return PSZ_SUCCESS;
}

int psz_amd_set_layout(psz_resource* m, int layout)
{
  Pipeline* p = cusz_amd::P(m);
  if (!p) return PSZ_AMD_ERR_INVALID_ARG;
  if (layout != PSZ_AMD_LAYOUT_BRICK && layout != PSZ_AMD_LAYOUT_REFERENCE && layout != PSZ_AMD_LAYOUT_BRICK_FORCE)
    return PSZ_AMD_ERR_INVALID_ARG;
  p->layout = layout == PSZ_AMD_LAYOUT_REFERENCE ? PSZ_AMD_LAYOUT_REFERENCE : PSZ_AMD_LAYOUT_BRICK;
  p->layout_set = layout == PSZ_AMD_LAYOUT_BRICK_FORCE;  // BRICK keeps the small-2-D default
  return PSZ_SUCCESS;
}

int psz_amd_decode_codes(psz_resource* m, uint8_t* in)
{
  Pipeline* p = cusz_amd::P(m);
  if (!p || !in) return PSZ_AMD_ERR_INVALID_ARG;
  return p->decode_codes(m->header, in);
}

const char* psz_amd_version(void) { return "cusz_amd 0.1 (gfx950)"; }

int psz_amd_last_create_status(void) { return g_create_status; }

int psz_amd_build_book_device(const uint32_t* IN_d_hist, int bklen, uint32_t smooth, uint32_t* OUT_d_book,
                              uint8_t* OUT_d_revbook, void* stream)
{
  if (!IN_d_hist || !OUT_d_book || !OUT_d_revbook || bklen < 1 || bklen > 1024) return PSZ_AMD_ERR_INVALID_ARG;
  CUSZ_AMD_HIP_CHECK((hipError_t)cusz_amd::launch_book_device(IN_d_hist, bklen, smooth, OUT_d_book, OUT_d_revbook,
                                                                (hipStream_t)stream));
  return PSZ_SUCCESS;
}

// internal: the older API passes a stream per call (cusz.h psz_compress/psz_decompress)
int cusz_amd_set_stream(psz_resource* m, void* stream)
{
  Pipeline* p = cusz_amd::P(m);
  if (!p) return PSZ_AMD_ERR_INVALID_ARG;
  p->stream = (hipStream_t)stream;
  m->stream = stream;
  return PSZ_SUCCESS;
}

// =========================================================================================
// header / phf helpers (psz/src/utils/header.c:9-30, codec/hf/src/libphf.cc:26-76)
// =========================================================================================

psz_len pszheader_len(psz_header* h) { return h->len; }
size_t pszheader_len_linear(psz_header* h) { return h->len.x * h->len.y * h->len.z; }
size_t pszheader_segments(psz_header* h)
{
  (void)h;
  return sizeof(psz_header);
}
size_t pszheader_filesize(psz_header* h) { return h->entry[PSZHEADER_ENC_PASS2_END]; }
size_t pszheader_uncompressed_len(psz_header* h) { return pszheader_len_linear(h); }
size_t pszheader_compressed_bytes(psz_header* h) { return pszheader_filesize(h); }

uint32_t phf_encoded_bytes(phf_header* h) { return h->entry[PHFHEADER_END]; }

size_t phf_coarse_tune_sublen(size_t len)
{
  int dev = 0, s, p;
  (void)hipGetDevice(&dev);
  cusz_amd::tune_chunking(len, dev, &s, &p);
  return (size_t)s;
}

void phf_coarse_tune(size_t len, int* sublen, int* pardeg)
{
  int dev = 0;
  (void)hipGetDevice(&dev);
  cusz_amd::tune_chunking(len, dev, sublen, pardeg);
}

size_t phf_reverse_book_bytes(u2 bklen, size_t BK_UNIT_BYTES, size_t SYM_BYTES)
{
  return BK_UNIT_BYTES * (2 * BK_UNIT_BYTES * 8) + SYM_BYTES * bklen;
}

void phf_version(void) { std::printf("\n///  cusz_amd HF (gfx950) build\n"); }
void phf_versioninfo(void) { phf_version(); }

}  // extern "C"
