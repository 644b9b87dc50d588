// oracle/ref_shim.cc -- TEST INFRASTRUCTURE ONLY.
//
// A thin extern "C" wrapper that is compiled together with the reference's own
// CPU translation units *where they lie* under /root/reference (see
// oracle/Makefile, target `ref`).  Nothing from the reference is copied into
// this repository; this file only calls the reference's templates/functions so
// that the pytest suite (and bench.py's cpu_baseline leg) can drive them via
// ctypes.  The product path never loads the resulting oracle/_ref/libpszref.so.
//
// Wrapped reference entry points:
//   psz::module::CPU_c_lorenzo_nd_with_outlier<f4,false,u2>::kernel   psz/src/kernel/lrz.seq.cc:35-55
//   psz::module::CPU_x_lorenzo_nd<f4,false,u2>::kernel                psz/src/kernel/lrz.seq.cc:57-77
//   psz::module::CPU_c_lorenzo_nd_with_outlier<f4,true,u2>::kernel    psz/src/kernel/lrz.seq.cc:82 (ZigZag)
//   psz::KERNEL_SEQ_c_lorenzo_3d1l<f8,false,u2>                       psz/src/kernel/detail/lrz.seq.inl:351-406
//   psz::KERNEL_SEQ_{c,x}_lorenzo_{1,2,3}d1l                          psz/src/kernel/detail/lrz.seq.inl:154-545
//   psz::module::SEQ_histogram_generic<u2>                            psz/src/kernel/hist_generic.seq.cc:17-30
//   phf_CPU_build_canonized_codebook_v2<u2,u4>                        codec/hf/src/hf_bk.seq.cc:72-145
//   psz::module::CPU_scatter<f4,u4>::kernel_v2                        psz/src/kernel/spvn.seq.cc:19-29

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>
#include <cstdint>
#include <cstring>
#include <memory>

// the 3-D template, instantiated below for f8; its file-scope helper object `div3` is renamed
// here so that it does not collide with lrz.seq.cc's copy at link time
#define div3 ref_shim_div3
#include "kernel/detail/lrz.seq.inl"
#undef div3

#include "c_type.h"
#include "hf_impl.hh"
#include "kernel/hist.hh"
#include "kernel/predictor.hh"
#include "kernel/spvn.hh"
#include "mem/cxx_sp_cpu.h"

namespace {
using Cell = _portable::compact_cell<f4, u4>;

// Points the reference CPU Lorenzo kernels predict (and may append as outliers): every point of
// every partial tile, i.e. the field padded to whole tiles of the dimension's block size
// (lrz.seq.inl:154/250/354: 256, 16 x 16, 8 x 8 x 8).
size_t padded_points(size_t x, size_t y, size_t z)
{
  auto up = [](size_t v, size_t m) { return (v + m - 1) / m * m; };
  if (z > 1) return up(x, 8) * up(y, 8) * up(z, 8);
  if (y > 1) return up(x, 16) * up(y, 16);
  return up(x, 256);
}
}  // namespace

extern "C" {

// Reference CPU Lorenzo compress (NOT error-bounded: no round(); BLK 256/16/8).
// Outliers are returned in the reference's sequential append order.
// Returns the outlier count, or UINT32_MAX when the kernel appended more than `ol_cap` cells (the
// reference does not bound-check: size `ol_cap` by the padded tile volume, pyoracle does).
uint32_t ref_c_lorenzo_f32(
    const float* in, size_t x, size_t y, size_t z, double eb, uint16_t radius, uint16_t* codes,
    float* ol_val, uint32_t* ol_idx, size_t ol_cap)
{
  auto outlier = std::make_unique<_portable::compact_CPU<f4, u4>>(ol_cap);
  psz_len len{x, y, z};
  psz::module::CPU_c_lorenzo_nd_with_outlier<f4, false, u2>::kernel(
      const_cast<float*>(in), len, codes, outlier.get(), eb, radius, nullptr);
  uint32_t n = outlier->num();
  if (n > ol_cap) return UINT32_MAX;
  for (uint32_t i = 0; i < n; i++) {
    ol_val[i] = outlier->val_idx(i).val;
    ol_idx[i] = outlier->val_idx(i).idx;
  }
  return n;
}

// ZigZag variant (the reference's own instantiation, lrz.seq.cc:82).
uint32_t ref_c_lorenzo_zz_f32(
    const float* in, size_t x, size_t y, size_t z, double eb, uint16_t radius, uint16_t* codes,
    float* ol_val, uint32_t* ol_idx, size_t ol_cap)
{
  auto outlier = std::make_unique<_portable::compact_CPU<f4, u4>>(ol_cap);
  psz_len len{x, y, z};
  psz::module::CPU_c_lorenzo_nd_with_outlier<f4, true, u2>::kernel(
      const_cast<float*>(in), len, codes, outlier.get(), eb, radius, nullptr);
  uint32_t n = outlier->num();
  if (n > ol_cap) return UINT32_MAX;
  for (uint32_t i = 0; i < n; i++) {
    ol_val[i] = outlier->val_idx(i).val;
    ol_idx[i] = outlier->val_idx(i).idx;
  }
  return n;
}

// 3-D f64: the reference's template instantiated for double, called the way
// CPU_c_lorenzo_nd_with_outlier calls it (lrz.seq.cc:35-55).
uint32_t ref_c_lorenzo3d_f64(
    const double* in, size_t x, size_t y, size_t z, double eb, uint16_t radius, uint16_t* codes,
    float* ol_val, uint32_t* ol_idx, size_t ol_cap)
{
  auto outlier = std::make_unique<_portable::compact_CPU<f8>>(ol_cap);
  psz_len len{x, y, z};
  auto leap3 = psz_len{1, x, x * y};
  psz::KERNEL_SEQ_c_lorenzo_3d1l<f8, false, u2>(
      const_cast<double*>(in), len, leap3, radius, 1 / (eb * 2), codes, outlier.get());
  uint32_t n = outlier->num();
  if (n > ol_cap) return UINT32_MAX;
  for (uint32_t i = 0; i < n; i++) {
    ol_val[i] = (float)outlier->val_idx(i).val;
    ol_idx[i] = outlier->val_idx(i).idx;
  }
  return n;
}

// Reference CPU Lorenzo decompress. `out` must hold the scattered outlier
// values and zeros elsewhere (reference convention, see lrz.seq.inl x-kernels).
void ref_x_lorenzo_f32(
    const uint16_t* codes, float* outlier_plane, float* out, size_t x, size_t y, size_t z,
    double eb, uint16_t radius)
{
  psz_len len{x, y, z};
  psz::module::CPU_x_lorenzo_nd<f4, false, u2>::kernel(
      const_cast<uint16_t*>(codes), outlier_plane, out, len, eb, radius, nullptr);
}

void ref_scatter_f32(const float* val, const uint32_t* idx, uint32_t n, float* out)
{
  auto cells = std::make_unique<Cell[]>(n ? n : 1);
  for (uint32_t i = 0; i < n; i++) cells[i] = Cell{val[i], idx[i]};
  psz::module::CPU_scatter<f4, u4>::kernel_v2(cells.get(), (int)n, out);
}

void ref_histogram_u2(const uint16_t* codes, size_t n, uint32_t* hist, uint16_t bklen)
{
  memset(hist, 0, sizeof(uint32_t) * bklen);
  psz::module::SEQ_histogram_generic<u2>(const_cast<uint16_t*>(codes), n, hist, bklen, nullptr);
}

// book: u32[bklen]; revbook: 4*64 + 2*bklen bytes (u2 symbols)
int ref_build_codebook_u2(const uint32_t* hist, int bklen, uint32_t* book, uint8_t* revbook)
{
  int rvbk_bytes = (int)phf_reverse_book_bytes(bklen, 4, sizeof(u2));
  memset(revbook, 0, rvbk_bytes);
  try {
    phf_CPU_build_canonized_codebook_v2<u2, u4>(
        const_cast<uint32_t*>(hist), bklen, book, revbook, rvbk_bytes, nullptr);
  }
  catch (...) {
    return -1;
  }
  return rvbk_bytes;
}

// Timing helpers for the CPU baseline leg: the reference CPU compress stages (c_lorenzo,
// histogram, codebook, x_lorenzo) on one field, milliseconds per stage in ms[0..3].  Every
// buffer is allocated and zeroed before the stage clocks start.
}  // extern "C"

namespace {

struct StageRun {
  size_t x, y, z, n, npad;
  std::unique_ptr<uint16_t[]> codes;
  std::unique_ptr<_portable::compact_CPU<f4, u4>> outlier;
  std::unique_ptr<uint32_t[]> hist, book;
  std::unique_ptr<uint8_t[]> revbook;
  std::unique_ptr<float[]> xdata;
  int rvbk_bytes;
  uint16_t radius;

  StageRun(size_t x_, size_t y_, size_t z_, uint16_t radius_) : x(x_), y(y_), z(z_), radius(radius_)
  {
    n = x * y * z;
    // The reference predicts every point of a partial tile, stale buffer contents included, and
    // may record outliers at indices past the field (lrz.seq.inl:266-284: no boundary check
    // before the outlier append); CPU_scatter then writes them.  Size the outlier list and the
    // scatter target for the largest such index (x < 256-, y < 16-, z < 8-multiples).
    auto up = [](size_t v, size_t m) { return (v + m - 1) / m * m; };
    const size_t ry = y == 1 ? 1 : up(y, 16), rz = z == 1 ? 1 : up(z, 8);
    npad = up(x, 256) + ry * x + rz * x * y;
    codes = std::make_unique<uint16_t[]>(n);
    memset(codes.get(), 0, sizeof(uint16_t) * n);  // pages faulted in before the clocks
    // the outlier list holds every predicted point (a count bound, unlike npad's index bound)
    outlier = std::make_unique<_portable::compact_CPU<f4, u4>>(std::max(npad, padded_points(x, y, z)));
    hist = std::make_unique<uint32_t[]>(2 * radius);
    book = std::make_unique<uint32_t[]>(2 * radius);
    rvbk_bytes = (int)phf_reverse_book_bytes(2 * radius, 4, sizeof(u2));
    revbook = std::make_unique<uint8_t[]>(rvbk_bytes);
    xdata = std::make_unique<float[]>(npad);
    memset(hist.get(), 0, sizeof(uint32_t) * 2 * radius);
    memset(xdata.get(), 0, sizeof(float) * npad);
  }

  // c_lorenzo, histogram, codebook; then the outlier scatter (untimed) and x_lorenzo
  void run(const float* in, double eb, double* ms, bool with_book)
  {
    using clk = std::chrono::steady_clock;
    auto ms_since = [](clk::time_point t0) {
      return std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    };
    psz_len len{x, y, z};
    auto t0 = clk::now();
    psz::module::CPU_c_lorenzo_nd_with_outlier<f4, false, u2>::kernel(
        const_cast<float*>(in), len, codes.get(), outlier.get(), eb, radius, nullptr);
    ms[0] = ms_since(t0);
    t0 = clk::now();
    psz::module::SEQ_histogram_generic<u2>(codes.get(), n, hist.get(), 2 * radius, nullptr);
    ms[1] = ms_since(t0);
    ms[2] = 0;
    if (with_book) {
      t0 = clk::now();
      phf_CPU_build_canonized_codebook_v2<u2, u4>(
          hist.get(), 2 * radius, book.get(), revbook.get(), rvbk_bytes, nullptr);
      ms[2] = ms_since(t0);
    }
    psz::module::CPU_scatter<f4, u4>::kernel_v2(outlier->val_idx(), outlier->num(), xdata.get());
    t0 = clk::now();
    psz::module::CPU_x_lorenzo_nd<f4, false, u2>::kernel(
        codes.get(), xdata.get(), xdata.get(), len, eb, radius, nullptr);
    ms[3] = ms_since(t0);
  }
};

}  // namespace

extern "C" {

void ref_time_stages_f32(
    const float* in, size_t x, size_t y, size_t z, double eb, uint16_t radius, double* ms)
{
  StageRun r(x, y, z, radius);
  r.run(in, eb, ms, true);
}

// All-core variant: slab s (element offset off[s], dims dims[3s..3s+2]) on its own thread.
// Every thread allocates and zeroes its buffers, then all start the stage clocks together
// (barrier) and free nothing until all are done, so no thread's mmap/munmap or page faults
// stall another's timed stages.  ms[4s..4s+3] per slab; returns the wall time in ms of the
// concurrent region (the slowest thread's c_lorenzo + histogram + scatter + x_lorenzo).
double ref_time_stages_par_f32(
    const float* in, int nslab, const size_t* off, const size_t* dims, double eb, uint16_t radius,
    double* ms)
{
  std::vector<std::unique_ptr<StageRun>> runs(nslab);
  std::mutex mu;
  std::condition_variable cv;
  int ready = 0, done = 0;
  std::chrono::steady_clock::time_point t0, t1;
  std::vector<std::thread> th;
  for (int s = 0; s < nslab; s++)
    th.emplace_back([&, s] {
      runs[s] = std::make_unique<StageRun>(dims[3 * s], dims[3 * s + 1], dims[3 * s + 2], radius);
      {
        std::unique_lock<std::mutex> lk(mu);
        if (++ready == nslab) {
          t0 = std::chrono::steady_clock::now();
          cv.notify_all();
        }
        else
          cv.wait(lk, [&] { return ready == nslab; });
      }
      runs[s]->run(in + off[s], eb, ms + 4 * s, false);
      {
        std::unique_lock<std::mutex> lk(mu);
        if (++done == nslab) {
          t1 = std::chrono::steady_clock::now();
          cv.notify_all();
        }
        else
          cv.wait(lk, [&] { return done == nslab; });
      }
    });
  for (auto& t : th) t.join();
  return std::chrono::duration<double, std::milli>(t1 - t0).count();
}

}  // extern "C"
