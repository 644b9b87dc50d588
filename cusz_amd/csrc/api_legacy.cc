// cusz_amd/csrc/api_legacy.cc -- context helpers, argv parsing and the older cusz.h API.
//
// pszctx_* / CLI_* follow psz/src/utils/context.cc:458-860 (defaults :779-826: Rel mode,
// eb 0.1, radius 512, Lorenzo + generic histogram + Huffman); argv parsing accepts the
// same flags as the reference `cusz` (context.cc:469-684) but reports errors through
// ctx->last_error instead of exit()/throw.  psz_create*/psz_compress/psz_decompress follow
// psz/src/libcusz.cc:29-214 and run on the same device pipeline as cusz_rev1.h.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "cusz.h"
#include "cusz_amd.h"
#include "cusz_rev1.h"
#include "hf.h"

namespace {

void fill_default_header(psz_header* h)
{
  std::memset(h, 0, sizeof(*h));
  h->dtype = F4;
  h->pipeline = psz_pipeline{Lorenzo, HistogramGeneric, Huffman, NullCodec};
  h->rc.mode = Rel;
  h->rc.eb = 0.1;
  h->rc.radius = 512;
  h->vle_sublen = 512;
  h->vle_pardeg = -1;
  h->len = psz_len{1, 1, 1};
  h->intp_param = make_default_params();
}

std::vector<std::string> split_dims(const char* s)
{  // context.cc:266-288: first delimiter found among x * - , m
  std::string str(s);
  std::vector<std::string> out;
  for (char d : {'x', '*', '-', ',', 'm'}) {
    if (str.find(d) == std::string::npos) continue;
    size_t b = 0;
    while (true) {
      size_t e = str.find(d, b);
      out.push_back(str.substr(b, e == std::string::npos ? std::string::npos : e - b));
      if (e == std::string::npos) break;
      b = e + 1;
    }
    return out;
  }
  out.push_back(str);
  return out;
}

void copy_str(char* dst, size_t cap, const char* src)
{
  std::snprintf(dst, cap, "%s", src);
}

}  // namespace

extern "C" {

void psz_version(void) { std::printf("\n///  cusz_amd (MI355X / gfx950 native cuSZ hot path) 0.1\n"); }

void psz_versioninfo(void)
{
  psz_version();
  int dev = 0;
  hipDeviceProp_t prop;
  if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
    std::printf("device %d: %s, %d CUs, %.1f GiB\n", dev, prop.gcnArchName, prop.multiProcessorCount,
                prop.totalGlobalMem / 1073741824.0);
}

psz_ctx* pszctx_default_values(void)
{
  auto* ctx = new (std::nothrow) psz_ctx;
  if (!ctx) return nullptr;
  std::memset(ctx, 0, sizeof(*ctx));
  ctx->header = new (std::nothrow) psz_header;
  ctx->cli = new (std::nothrow) psz_cli_config;
  if (!ctx->header || !ctx->cli) {
    delete ctx->header;
    delete ctx->cli;
    delete ctx;
    return nullptr;
  }
  fill_default_header(ctx->header);
  std::memset(ctx->cli, 0, sizeof(psz_cli_config));
  ctx->device = AMDGPU;
  ctx->dict_size = 1024;
  ctx->len_linear = 1;
  ctx->ndim = -1;
  return ctx;
}

void pszctx_set_default_values(psz_ctx* ctx)
{
  psz_ctx* d = pszctx_default_values();
  if (!d) return;
  std::memcpy(ctx, d, sizeof(psz_ctx));
  delete d;  // header/cli ownership moved into ctx
}

psz_ctx* pszctx_minimal_workset(psz_dtype const dtype, psz_predictor const predictor, int const quantizer_radius,
                                psz_codec const codec)
{
  psz_ctx* ws = pszctx_default_values();
  if (!ws) return nullptr;
  ws->header->dtype = dtype;
  ws->header->pipeline.predictor = predictor;
  ws->header->pipeline.codec1 = codec;
  ws->dict_size = (uint16_t)(quantizer_radius * 2);
  ws->header->rc.radius = (uint16_t)quantizer_radius;
  return ws;
}

void pszctx_set_rawlen(psz_ctx* ctx, size_t x, size_t y, size_t z)
{
  ctx->header->len = psz_len{x, y, z};
  ctx->ndim = z == 1 ? (y == 1 ? 1 : 2) : 3;
  ctx->len_linear = x * y * z;
  if (ctx->len_linear <= 1) ctx->last_error = PSZ_ABORT_UNSUPPORTED_DIMENSION;
}

void pszctx_set_len(psz_ctx* ctx, psz_len3 len) { pszctx_set_rawlen(ctx, len.x, len.y, len.z); }

psz_len3 pszctx_get_len3(psz_ctx* ctx) { return ctx->header->len; }

// Parse cusz-style argv into ctx; on error sets ctx->last_error (never exits/throws).
void pszctx_create_from_argv(psz_ctx* ctx, int const argc, char** const argv)
{
  auto need = [&](int i) -> bool {
    if (i + 1 >= argc) {
      std::fprintf(stderr, "[cusz] missing value after %s\n", argv[i]);
      ctx->last_error = (psz_error_status)PSZ_AMD_ERR_INVALID_ARG;
      return false;
    }
    return true;
  };
  auto is = [](const char* a, std::initializer_list<const char*> names) {
    for (auto n : names)
      if (std::strcmp(a, n) == 0) return true;
    return false;
  };
  for (int i = 1; i < argc; i++) {
    const char* a = argv[i];
    if (is(a, {"-m", "--mode"})) {
      if (!need(i)) return;
      std::string v = argv[++i];
      ctx->header->rc.mode = (v == "r2r" || v == "rel") ? Rel : Abs;
      ctx->cli->rel_range_scan = ctx->header->rc.mode == Rel;
      copy_str(ctx->cli->char_mode, sizeof(ctx->cli->char_mode), v.c_str());
    }
    else if (is(a, {"-e", "--eb", "--error-bound"})) {
      if (!need(i)) return;
      ctx->header->rc.eb = std::strtod(argv[++i], nullptr);
      copy_str(ctx->cli->char_meta_eb, sizeof(ctx->cli->char_meta_eb), argv[i]);
    }
    else if (is(a, {"-p", "--pred", "--predictor"})) {
      if (!need(i)) return;
      std::string v = argv[++i];
      copy_str(ctx->cli->char_predictor_name, sizeof(ctx->cli->char_predictor_name), v.c_str());
      if (v == "spline" || v == "spline3" || v == "spl") ctx->header->pipeline.predictor = Spline;
      else if (v == "lorenzo-zigzag" || v == "lrz-zz") ctx->header->pipeline.predictor = LorenzoZigZag;
      else if (v == "lorenzo-proto" || v == "lrz-proto") ctx->header->pipeline.predictor = LorenzoProto;
      else ctx->header->pipeline.predictor = Lorenzo;
    }
    else if (is(a, {"--hist", "--histogram"})) {
      if (!need(i)) return;
      std::string v = argv[++i];
      copy_str(ctx->cli->char_hist_name, sizeof(ctx->cli->char_hist_name), v.c_str());
      ctx->header->pipeline.hist = v == "sparse" ? HistogramSparse : HistogramGeneric;
    }
    else if (is(a, {"-c1", "--codec", "--codec1"})) {
      if (!need(i)) return;
      std::string v = argv[++i];
      copy_str(ctx->cli->char_codec1_name, sizeof(ctx->cli->char_codec1_name), v.c_str());
      ctx->header->pipeline.codec1 = v == "fzgcodec" ? FZCodec : Huffman;
    }
    else if (is(a, {"-t", "--type", "--dtype"})) {
      if (!need(i)) return;
      std::string v = argv[++i];
      if (v == "f32" || v == "f4") ctx->header->dtype = F4;
      else if (v == "f64" || v == "f8") ctx->header->dtype = F8;
    }
    else if (is(a, {"-i", "--input"})) {
      if (!need(i)) return;
      copy_str(ctx->cli->file_input, sizeof(ctx->cli->file_input), argv[++i]);
    }
    else if (is(a, {"-l", "--len", "--xyz", "--dim3"})) {
      if (!need(i)) return;
      auto d = split_dims(argv[++i]);
      size_t l[3] = {1, 1, 1};
      for (size_t k = 0; k < d.size() && k < 3; k++) l[k] = std::strtoull(d[k].c_str(), nullptr, 10);
      ctx->header->len = psz_len{l[0], l[1], l[2]};
      ctx->ndim = (int)d.size();
      ctx->len_linear = l[0] * l[1] * l[2];
    }
    else if (is(a, {"--math-order", "--zyx", "--slowest-to-fastest"})) {
      if (!need(i)) return;
      auto d = split_dims(argv[++i]);
      size_t l[3] = {1, 1, 1};
      const int nd = (int)d.size();
      for (int k = 0; k < nd && k < 3; k++) l[k] = std::strtoull(d[nd - 1 - k].c_str(), nullptr, 10);
      ctx->header->len = psz_len{l[0], l[1], l[2]};
      ctx->ndim = nd;
      ctx->len_linear = l[0] * l[1] * l[2];
    }
    else if (is(a, {"-z", "--zip", "--compress"}))
      ctx->cli->task_construct = true;
    else if (is(a, {"-x", "--unzip", "--decompress"}))
      ctx->cli->task_reconstruct = true;
    else if (is(a, {"--verbose"}))
      ctx->cli->verbose = true;
    else if (is(a, {"-R", "--report"})) {
      if (!need(i)) return;
      std::string v = argv[++i];
      ctx->cli->report_time = v.find("time") != std::string::npos;
      ctx->cli->report_cr = v.find("cr") != std::string::npos;
    }
    else if (is(a, {"--dump"})) {
      if (!need(i)) return;
      std::string v = argv[++i];
      ctx->cli->dump_quantcode = v.find("quant") != std::string::npos;
      ctx->cli->dump_hist = v.find("hist") != std::string::npos;
    }
    else if (is(a, {"-S", "-X", "--skip", "--exclude"})) {
      if (!need(i)) return;
      std::string v = argv[++i];
      ctx->cli->skip_hf = v.find("huffman") != std::string::npos;
      ctx->cli->skip_tofile = v.find("write2disk") != std::string::npos;
    }
    else if (is(a, {"--origin", "--compare"})) {
      if (!need(i)) return;
      copy_str(ctx->cli->file_compare, sizeof(ctx->cli->file_compare), argv[++i]);
    }
    else if (is(a, {"-s", "--scheme"})) {
      if (!need(i)) return;
      std::string v = argv[++i];
      if (v == "cr" || v == "CR") ctx->header->pipeline.codec1 = Huffman;
    }
    else if (is(a, {"-a", "--auto"})) {
      if (!need(i)) return;
      std::string v = argv[++i];
      ctx->header->intp_param.auto_tuning =
          (v == "rd-first" || v == "RD-first") ? 6 : (v == "cr-first" || v == "CR-first") ? 3 : (uint8_t)std::atoi(v.c_str());
    }
    else {
      std::fprintf(stderr, "[cusz] invalid option at position %d: %s\n", i, a);
      ctx->last_error = (psz_error_status)PSZ_AMD_ERR_INVALID_ARG;
      return;
    }
  }
  ctx->dict_size = (uint16_t)(ctx->header->rc.radius * 2);
}

psz_resource* psz_create_resource_manager_from_CLI(int argc, char** argv, void* stream)
{
  psz_ctx* ctx = pszctx_default_values();
  if (!ctx) return nullptr;
  pszctx_create_from_argv(ctx, argc, argv);
  psz_resource* m = nullptr;
  if (ctx->last_error == PSZ_SUCCESS)
    m = psz_create_resource_manager(ctx->header->dtype, ctx->header->len, ctx->header->pipeline, stream);
  if (m) {
    m->header->rc = ctx->header->rc;
    m->cli = ctx->cli;
    ctx->cli = nullptr;
  }
  delete ctx->cli;
  delete ctx->header;
  delete ctx;
  return m;
}

unsigned int CLI_x(psz_args* a) { return (unsigned)a->header->len.x; }
unsigned int CLI_y(psz_args* a) { return (unsigned)a->header->len.y; }
unsigned int CLI_z(psz_args* a) { return (unsigned)a->header->len.z; }
unsigned int CLI_w(psz_args* a)
{
  (void)a;
  return 1;
}
unsigned short CLI_radius(psz_args* a) { return a->header->rc.radius; }
unsigned short CLI_bklen(psz_args* a) { return (unsigned short)(a->header->rc.radius * 2); }
psz_dtype CLI_dtype(psz_args* a) { return a->header->dtype; }
psz_predictor CLI_predictor(psz_args* a) { return a->header->pipeline.predictor; }
psz_hist CLI_hist(psz_args* a) { return a->header->pipeline.hist; }
psz_codec CLI_codec1(psz_args* a) { return a->header->pipeline.codec1; }
psz_codec CLI_codec2(psz_args* a) { return a->header->pipeline.codec2; }
psz_mode CLI_mode(psz_args* a) { return a->header->rc.mode; }
double CLI_eb(psz_args* a) { return a->header->rc.eb; }
psz_interp_params* CLI_interp_params(psz_ctx* ctx) { return &ctx->header->intp_param; }

// ---- older compressor-object API ---------------------------------------------------------

static psz_compressor* wrap(psz_ctx* ctx)
{
  auto* comp = new (std::nothrow) psz_compressor;
  if (!comp) return nullptr;
  comp->ctx = ctx;
  comp->last_error = PSZ_SUCCESS;
  comp->mem = nullptr;
  comp->compressor = nullptr;
  if (!ctx) {
    comp->last_error = (psz_error_status)PSZ_AMD_ERR_INVALID_ARG;
    return comp;
  }
  if (ctx->header->dtype != F4 && ctx->header->dtype != F8) {
    comp->last_error = PSZ_ABORT_UNSUPPORTED_TYPE;
    return comp;
  }
  phf_coarse_tune(ctx->len_linear, &ctx->header->vle_sublen, &ctx->header->vle_pardeg);
  psz_resource* m = psz_create_resource_manager_from_header(ctx->header, nullptr);
  if (!m) comp->last_error = (psz_error_status)PSZ_AMD_ERR_DEVICE;  // allocation or runtime failure
  comp->compressor = m;
  return comp;
}

psz_compressor* psz_create(psz_dtype const dtype, psz_len3 const len, psz_predictor const predictor,
                           int const quantizer_radius, psz_codec const codec)
{
  psz_ctx* ctx = pszctx_minimal_workset(dtype, predictor, quantizer_radius, codec);
  if (ctx) pszctx_set_len(ctx, len);
  return wrap(ctx);
}

psz_compressor* psz_create_default(psz_dtype const dtype, psz_len3 const len)
{
  psz_ctx* ctx = pszctx_default_values();
  if (ctx) ctx->header->dtype = dtype, pszctx_set_len(ctx, len);
  return wrap(ctx);
}

psz_compressor* psz_create_from_context(psz_ctx* const ctx, psz_len3 const len)
{
  pszctx_set_len(ctx, len);
  return wrap(ctx);
}

psz_compressor* psz_create_from_header(psz_header* const h)
{
  psz_ctx* ctx = pszctx_default_values();
  if (!ctx) return wrap(nullptr);
  *ctx->header = *h;
  ctx->len_linear = h->len.x * h->len.y * h->len.z;
  ctx->dict_size = (uint16_t)(h->rc.radius * 2);
  return wrap(ctx);
}

pszerror psz_release(psz_compressor* comp)
{
  if (!comp) return PSZ_SUCCESS;
  psz_release_resource((psz_resource*)comp->compressor);
  if (comp->ctx) {
    delete comp->ctx->cli;
    delete comp->ctx->header;
    delete comp->ctx;
  }
  delete comp;
  return PSZ_SUCCESS;
}

int cusz_amd_set_stream(psz_resource* m, void* stream);

pszerror psz_compress(psz_compressor* comp, void* d_in, psz_len3 const in_len3, double const eb,
                      psz_mode const mode, uint8_t** d_compressed, size_t* comp_bytes, psz_header* header,
                      void* record, void* stream)
{
  (void)record;
  if (!comp || !comp->compressor) return (pszerror)PSZ_AMD_ERR_INVALID_ARG;
  auto* m = (psz_resource*)comp->compressor;
  if (in_len3.x != m->header->len.x || in_len3.y != m->header->len.y || in_len3.z != m->header->len.z)
    return PSZ_ABORT_UNSUPPORTED_DIMENSION;
  cusz_amd_set_stream(m, stream);
  psz_rc2 rc{mode, eb, comp->ctx->header->rc.radius};
  int s = comp->ctx->header->dtype == F4
              ? psz_compress_float(m, rc, (float*)d_in, header, d_compressed, comp_bytes)
              : psz_compress_double(m, rc, (double*)d_in, header, d_compressed, comp_bytes);
  *comp->ctx->header = *m->header;  // psz_decompress reads it back (also when header == NULL)
  comp->last_error = (psz_error_status)s;
  return (pszerror)s;
}

pszerror psz_decompress(psz_compressor* comp, uint8_t* d_compressed, size_t const comp_len, void* d_decompressed,
                        psz_len3 const decomp_len, void* record, void* stream)
{
  (void)record;
  (void)decomp_len;
  if (!comp || !comp->compressor) return (pszerror)PSZ_AMD_ERR_INVALID_ARG;
  auto* m = (psz_resource*)comp->compressor;
  cusz_amd_set_stream(m, stream);
  psz_modify_resource_manager_from_header(m, comp->ctx->header);
  int s = comp->ctx->header->dtype == F4
              ? psz_decompress_float(m, d_compressed, comp_len, (float*)d_decompressed)
              : psz_decompress_double(m, d_compressed, comp_len, (double*)d_decompressed);
  comp->last_error = (psz_error_status)s;
  return (pszerror)s;
}

pszerror psz_clear_buffer(psz_compressor* comp)
{
  (void)comp;  // every call resets its own state
  return PSZ_SUCCESS;
}

void* psz_make_timerecord(void) { return nullptr; }
void psz_review_comp_time_breakdown(void* r, psz_header* h) { (void)r, (void)h; }
void psz_review_comp_time_from_header(psz_header* h) { (void)h; }
void psz_review_decomp_time_from_header(psz_header* h) { (void)h; }
void psz_review_compression(void* r, psz_header* h)
{
  (void)r;
  const size_t in = (h->len.x * h->len.y * h->len.z) * (h->dtype == F8 ? 8 : 4);
  std::printf("compression ratio: %.3f (%zu -> %u bytes, %zu outliers)\n",
              (double)in / h->entry[PSZHEADER_ENC_PASS2_END], in, h->entry[PSZHEADER_ENC_PASS2_END], h->splen);
}
void psz_review_decompression(void* r, size_t bytes) { (void)r, (void)bytes; }

}  // extern "C"
