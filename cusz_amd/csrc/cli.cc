// cusz_amd/csrc/cli.cc -- the `cusz` command line (drop-in for psz/src/cli/cli.cc:51-172).
//
//   cusz -t f32 -m abs -e 1e-4 -l 512x512x512 -z -i field.f32      -> field.f32.cusza
//   cusz -x -i field.f32.cusza [--origin field.f32]                -> field.f32.cuszx
//
// Archive file = the device archive verbatim (this build writes the 176-B psz_header into
// the device archive itself; the reference patches it in on the host, cli.cc:112-118).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "cusz.h"
#include "cusz_amd.h"
#include "cusz_rev1.h"

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "[cusz] HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                       \
    }                                                                                 \
  } while (0)

static bool read_file(const char* path, std::vector<char>& buf)
{
  FILE* f = std::fopen(path, "rb");
  if (!f) return false;
  std::fseek(f, 0, SEEK_END);
  long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  buf.resize((size_t)n);
  bool ok = std::fread(buf.data(), 1, (size_t)n, f) == (size_t)n;
  std::fclose(f);
  return ok;
}

static bool write_file(const std::string& path, const void* p, size_t n)
{
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) return false;
  bool ok = std::fwrite(p, 1, n, f) == n;
  std::fclose(f);
  return ok;
}

static void usage()
{
  std::printf(
      "usage: cusz -z -t f32|f64 -m abs|rel|r2r -e EB -l X[xY[xZ]] -i FILE [-p lrz|lrz-zz] [-R time,cr]\n"
      "       cusz -x -i FILE.cusza [--origin FILE] [-R time] [-S write2disk]\n");
}

template <typename T>
static void quality(const T* a, const T* b, size_t n, double eb)
{
  double maxe = 0, mn = INFINITY, mx = -INFINITY, se = 0;
  for (size_t i = 0; i < n; i++) {
    double d = std::fabs((double)a[i] - (double)b[i]);
    maxe = d > maxe ? d : maxe;
    se += d * d;
    mn = a[i] < mn ? a[i] : mn;
    mx = a[i] > mx ? a[i] : mx;
  }
  const double rng = mx - mn, mse = se / (double)n;
  const double psnr = 20 * std::log10(rng) - 10 * std::log10(mse);
  std::printf("max-error %.6e (eb %.6e, %s), PSNR %.3f dB, NRMSE %.6e\n", maxe, eb,
              maxe <= eb * 1.001 ? "bounded" : "NOT bounded", psnr, std::sqrt(mse) / rng);
}

// --dump hist,quant (compressor.inl:507-529): the histogram u32[2r] and the quant codes
// u16[N] in index order, as <input>.<mode>_<eb>.bk_<2r>.{ht_u4,qt_u2}.  The codes are decoded
// back from the archive with the per-chunk decoder (chunk c holds codes [c sublen, (c+1)
// sublen) whatever the layout), so the dump is in index order for both layouts.
static int dump_internals(const psz_ctx* ctx, psz_resource* m, uint8_t* d_arch, size_t n)
{
  const psz_header* h = ctx->header;
  auto name = [&](const char* suffix, const char* t) {
    return std::string(ctx->cli->file_input) + "." + ctx->cli->char_mode + "_" + ctx->cli->char_meta_eb + ".bk_" +
           std::to_string(2 * h->rc.radius) + "." + suffix + "_" + t;
  };
  psz_amd_internals io;
  if (psz_amd_get_internals(m, &io) != PSZ_SUCCESS) return 1;
  if (ctx->cli->dump_hist) {
    std::vector<uint32_t> hist((size_t)io.bklen);
    CK(hipMemcpy(hist.data(), io.d_hist, hist.size() * 4, hipMemcpyDeviceToHost));
    if (!write_file(name("ht", "u4"), hist.data(), hist.size() * 4)) return 1;
  }
  if (ctx->cli->dump_quantcode) {
    std::printf("[psz::dump] dumping quantization codes to file: %s\n", name("qt", "u2").c_str());
    if (psz_amd_set_decoder(m, PSZ_AMD_DECODER_LANE) != PSZ_SUCCESS || psz_amd_decode_codes(m, d_arch) != PSZ_SUCCESS) {
      std::fprintf(stderr, "[cusz] cannot decode the archive for --dump quant\n");
      return 1;
    }
    std::vector<uint16_t> q(n);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(q.data(), io.d_quant_codes, n * 2, hipMemcpyDeviceToHost));
    if (!write_file(name("qt", "u2"), q.data(), n * 2)) return 1;
  }
  return 0;
}

int main(int argc, char** argv)
{
  if (argc == 1) {
    usage();
    return 0;
  }
  for (int i = 1; i < argc; i++) {
    if (!std::strcmp(argv[i], "-h") || !std::strcmp(argv[i], "--help")) return usage(), 0;
    if (!std::strcmp(argv[i], "-v") || !std::strcmp(argv[i], "--version")) return psz_version(), 0;
    if (!std::strcmp(argv[i], "-V") || !std::strcmp(argv[i], "--versioninfo")) return psz_versioninfo(), 0;
  }
  psz_ctx* ctx = pszctx_default_values();
  pszctx_create_from_argv(ctx, argc, argv);
  if (ctx->last_error != PSZ_SUCCESS) return usage(), 1;
  if (!ctx->cli->file_input[0] || (!ctx->cli->task_construct && !ctx->cli->task_reconstruct)) {
    std::fprintf(stderr, "[cusz] need -i FILE and -z or -x\n");
    return usage(), 1;
  }
  hipStream_t st;
  CK(hipStreamCreate(&st));
  using clk = std::chrono::steady_clock;

  if (ctx->cli->task_construct) {
    const psz_header* h = ctx->header;
    const size_t n = h->len.x * h->len.y * h->len.z;
    const size_t es = h->dtype == F8 ? 8 : 4;
    std::vector<char> in;
    if (!read_file(ctx->cli->file_input, in) || in.size() < n * es) {
      std::fprintf(stderr, "[cusz] cannot read %zu bytes from %s\n", n * es, ctx->cli->file_input);
      return 1;
    }
    void* d_in;
    CK(hipMalloc(&d_in, n * es));
    CK(hipMemcpy(d_in, in.data(), n * es, hipMemcpyHostToDevice));
    psz_resource* m = psz_create_resource_manager(h->dtype, h->len, h->pipeline, st);
    if (!m) return std::fprintf(stderr, "[cusz] cannot create resource manager\n"), 1;
    psz_amd_enable_timing(m, 1);
    psz_rc2 rc{h->rc.mode, h->rc.eb, h->rc.radius};
    psz_header out_h;
    uint8_t* d_arch;
    size_t bytes;
    auto t0 = clk::now();
    int s = h->dtype == F4 ? psz_compress_float(m, rc, (float*)d_in, &out_h, &d_arch, &bytes)
                           : psz_compress_double(m, rc, (double*)d_in, &out_h, &d_arch, &bytes);
    double wall = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    if (s != PSZ_SUCCESS && s != PSZ_WARN_RADIUS_TOO_LARGE) {
      std::fprintf(stderr, "[cusz] compress failed with status %d\n", s);
      return 1;
    }
    std::vector<char> arch(bytes);
    CK(hipMemcpy(arch.data(), d_arch, bytes, hipMemcpyDeviceToHost));
    std::string opath = std::string(ctx->cli->file_input) + ".cusza";
    if (!ctx->cli->skip_tofile && !write_file(opath, arch.data(), bytes)) return 1;
    float ms[PSZ_AMD_T_COUNT];
    psz_amd_stage_times(m, ms, PSZ_AMD_T_COUNT);
    if ((ctx->cli->dump_hist || ctx->cli->dump_quantcode) && dump_internals(ctx, m, d_arch, n)) return 1;
    std::printf("compressed %s -> %s: %zu -> %zu bytes, CR %.3f, outliers %zu\n", ctx->cli->file_input,
                opath.c_str(), n * es, bytes, (double)(n * es) / bytes, (size_t)out_h.splen);
    if (ctx->cli->report_time)
      std::printf("time: compress %.3f ms (device %.3f ms: predict %.3f, book %.3f, encode %.3f, finalize %.3f) "
                  "%.2f GB/s\n",
                  wall, ms[PSZ_AMD_T_COMPRESS], ms[PSZ_AMD_T_PREDICT], ms[PSZ_AMD_T_BOOK], ms[PSZ_AMD_T_ENCODE],
                  ms[PSZ_AMD_T_FINALIZE], n * es / (ms[PSZ_AMD_T_COMPRESS] * 1e6));
    psz_release_resource(m);
    CK(hipFree(d_in));
  }
  else {
    std::vector<char> arch;
    if (!read_file(ctx->cli->file_input, arch) || arch.size() < sizeof(psz_header)) {
      std::fprintf(stderr, "[cusz] cannot read archive %s\n", ctx->cli->file_input);
      return 1;
    }
    psz_header h;
    std::memcpy(&h, arch.data(), sizeof(h));
    const size_t n = h.len.x * h.len.y * h.len.z;
    const size_t es = h.dtype == F8 ? 8 : 4;
    uint8_t* d_arch;
    void* d_out;
    CK(hipMalloc(&d_arch, arch.size()));
    CK(hipMalloc(&d_out, n * es));
    CK(hipMemcpy(d_arch, arch.data(), arch.size(), hipMemcpyHostToDevice));
    psz_resource* m = psz_create_resource_manager_from_header(&h, st);
    if (!m) return std::fprintf(stderr, "[cusz] cannot create resource manager\n"), 1;
    psz_amd_enable_timing(m, 1);
    auto t0 = clk::now();
    int s = h.dtype == F4 ? psz_decompress_float(m, d_arch, arch.size(), (float*)d_out)
                          : psz_decompress_double(m, d_arch, arch.size(), (double*)d_out);
    CK(hipStreamSynchronize(st));
    double wall = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    if (s != PSZ_SUCCESS) return std::fprintf(stderr, "[cusz] decompress failed with status %d\n", s), 1;
    std::vector<char> out(n * es);
    CK(hipMemcpy(out.data(), d_out, n * es, hipMemcpyDeviceToHost));
    std::string base(ctx->cli->file_input);
    if (base.size() > 6 && base.substr(base.size() - 6) == ".cusza") base = base.substr(0, base.size() - 6);
    if (!ctx->cli->skip_tofile && !write_file(base + ".cuszx", out.data(), out.size())) return 1;
    float ms[PSZ_AMD_T_COUNT];
    psz_amd_stage_times(m, ms, PSZ_AMD_T_COUNT);
    std::printf("decompressed %s -> %s.cuszx (%zu bytes)\n", ctx->cli->file_input, base.c_str(), n * es);
    if (ctx->cli->report_time)
      std::printf("time: decompress %.3f ms (device %.3f ms) %.2f GB/s\n", wall, ms[PSZ_AMD_T_DECOMPRESS],
                  n * es / (ms[PSZ_AMD_T_DECOMPRESS] * 1e6));
    if (ctx->cli->file_compare[0]) {
      std::vector<char> orig;
      if (read_file(ctx->cli->file_compare, orig) && orig.size() >= n * es) {
        if (h.dtype == F4) quality((const float*)orig.data(), (const float*)out.data(), n, h.rc.eb);
        else quality((const double*)orig.data(), (const double*)out.data(), n, h.rc.eb);
      }
    }
    psz_release_resource(m);
    CK(hipFree(d_arch));
    CK(hipFree(d_out));
  }
  CK(hipStreamDestroy(st));
  return 0;
}
