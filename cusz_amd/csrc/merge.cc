// cusz_amd/csrc/merge.cc -- merge per-slab archives into one archive of the whole field (host).
//
// The multi-GPU path (the reference itself has no multi-GPU code) compresses
// tile-aligned slabs on separate GPUs with ONE codebook (built from the all-reduced histogram)
// and gathers the per-slab archives to a root rank.  Because prediction is tile-local and the
// chunking is the same, the slabs' Huffman chunks are exactly the chunks of a single-process
// run over the whole field, in the same order.  The merged archive is therefore the archive a
// single process would have written:
//   psz_header (176 B)  -- len = whole field, splen = sum, segment entries recomputed
//   phf header (64 B + pad to 128)  -- pardeg/original_len/total_nbit/total_ncell = sums
//   revbook             -- identical in every slab (shared codebook), written once
//   par_nbit            -- concatenated
//   par_entry           -- concatenated, each slab's entries rebased by the cells before it
//                          (the reference's exclusive scan of ncell, hf_buf.cc:199-211)
//   bitstream           -- concatenated
//   outlier cells       -- concatenated, idx rebased by the slab's element offset
//                          (compressor.inl:398-418 segment order)
// Pure host code over host buffers: no GPU is needed (the CPU tests call it through ctypes).
#include <cstdint>
#include <cstring>
#include <vector>

#include "cusz/header.h"
#include "cusz_amd.h"
#include "hf.h"

namespace {

struct Part {
  psz_header h;
  phf_header ph;
  const uint8_t* base;
  const uint8_t* phf;
  size_t n;
};

size_t rvbk_bytes(int bklen) { return 4 * 64 + 2 * (size_t)bklen; }

int ndim_of(psz_len l) { return l.z > 1 ? 3 : (l.y > 1 ? 2 : 1); }

// A slab of the field: same extents on every axis but the split (slowest) one, and -- unless it
// is the last slab -- a split extent that is a whole number of prediction tiles.
bool slab_shape_ok(psz_len s, psz_len f, bool last)
{
  switch (ndim_of(f)) {
    case 3: return s.x == f.x && s.y == f.y && s.z >= 1 && (last || s.z % 8 == 0);
    case 2: return s.x == f.x && s.z == 1 && s.y >= 1 && (last || s.y % 32 == 0);
    default: return s.y == 1 && s.z == 1 && s.x >= 1 && (last || s.x % 1024 == 0);
  }
}

// phf sections of one part (hf_buf.cc:199-211): monotonic offsets inside the segment the psz
// header gives the phf archive, tables sized by pardeg, bitstream by total_ncell, and every
// chunk's cells inside the bitstream.
bool phf_sections_ok(const Part& p, size_t seg)
{
  const uint32_t* pe = p.ph.entry;
  const size_t pd = (size_t)(p.ph.pardeg > 0 ? p.ph.pardeg : 0);
  if (p.ph.pardeg <= 0 || pe[PHFHEADER_END] > seg) return false;
  for (int k = 1; k <= PHFHEADER_END; k++)
    if (pe[k] < pe[k - 1]) return false;
  if (pe[PHFHEADER_RVBK] < sizeof(phf_header) || pe[PHFHEADER_PAR_NBIT] - pe[PHFHEADER_RVBK] != rvbk_bytes(p.ph.bklen) ||
      pe[PHFHEADER_PAR_ENTRY] - pe[PHFHEADER_PAR_NBIT] != 4 * pd ||
      pe[PHFHEADER_BITSTREAM] - pe[PHFHEADER_PAR_ENTRY] != 4 * pd ||
      pe[PHFHEADER_END] - pe[PHFHEADER_BITSTREAM] != 4 * p.ph.total_ncell)
    return false;
  const uint32_t* nb = reinterpret_cast<const uint32_t*>(p.phf + pe[PHFHEADER_PAR_NBIT]);
  const uint32_t* en = reinterpret_cast<const uint32_t*>(p.phf + pe[PHFHEADER_PAR_ENTRY]);
  for (size_t c = 0; c < pd; c++) {
    uint32_t nbit, ent;
    std::memcpy(&nbit, nb + c, 4);
    std::memcpy(&ent, en + c, 4);
    if ((uint64_t)ent + ((uint64_t)nbit + 31) / 32 > p.ph.total_ncell) return false;
  }
  return true;
}

}  // namespace

extern "C" int psz_amd_merge_archives(const uint8_t* const* parts, const size_t* part_bytes, int nparts,
                                      const size_t* elem_offsets, psz_len full_len, uint8_t* out, size_t out_cap,
                                      size_t* out_bytes)
{
  if (!parts || !part_bytes || nparts < 1 || !out_bytes) return PSZ_AMD_ERR_INVALID_ARG;
  std::vector<Part> P((size_t)nparts);
  size_t n_total = 0, splen = 0, ncell = 0, pardeg = 0;
  unsigned long long nbit = 0;
  for (int i = 0; i < nparts; i++) {
    Part& p = P[(size_t)i];
    if (!parts[i]) return PSZ_AMD_ERR_INVALID_ARG;
    if (part_bytes[i] < sizeof(psz_header)) return PSZ_AMD_ERR_BAD_ARCHIVE;
    std::memcpy(&p.h, parts[i], sizeof(psz_header));
    const uint32_t* e = p.h.entry;
    // anchors (spline) are per-slab 8^3 lattices: not mergeable by concatenation
    if (e[PSZHEADER_ANCHOR] != e[PSZHEADER_ENCODED]) return PSZ_ABORT_NO_SUCH_PREDICTOR;
    if (e[PSZHEADER_ENC_PASS2_END] > part_bytes[i] || e[PSZHEADER_ENCODED] + sizeof(phf_header) > part_bytes[i])
      return PSZ_AMD_ERR_BAD_ARCHIVE;
    for (int k = 1; k <= PSZHEADER_ENC_PASS2_END; k++)
      if (e[k] < e[k - 1]) return PSZ_AMD_ERR_BAD_ARCHIVE;
    p.base = parts[i];
    p.phf = parts[i] + e[PSZHEADER_ENCODED];
    std::memcpy(&p.ph, p.phf, sizeof(phf_header));
    p.n = p.h.len.x * p.h.len.y * p.h.len.z;
    // the part's own segments: outlier cells, phf sections inside the phf segment, chunk table
    if ((size_t)e[PSZHEADER_ENC_PASS1_END] - e[PSZHEADER_SPFMT] != 8 * p.h.splen) return PSZ_AMD_ERR_BAD_ARCHIVE;
    if (!phf_sections_ok(p, e[PSZHEADER_SPFMT] - e[PSZHEADER_ENCODED])) return PSZ_AMD_ERR_BAD_ARCHIVE;
    const Part& q = P[0];
    if (p.h.dtype != q.h.dtype || p.h.pipeline.predictor != q.h.pipeline.predictor || p.h.rc.radius != q.h.rc.radius ||
        p.h.rc.eb != q.h.rc.eb || p.ph.bklen != q.ph.bklen || p.ph.sublen != q.ph.sublen)
      return p.h.dtype != q.h.dtype ? PSZ_ABORT_UNSUPPORTED_TYPE : PSZ_AMD_ERR_INVALID_ARG;  // parts of different runs
    const size_t rv = rvbk_bytes(p.ph.bklen);
    if (p.ph.entry[PHFHEADER_END] + e[PSZHEADER_ENCODED] > part_bytes[i]) return PSZ_AMD_ERR_BAD_ARCHIVE;
    if (std::memcmp(p.phf + PHFHEADER_FORCED_ALIGN, q.phf + PHFHEADER_FORCED_ALIGN, rv) != 0)
      return PSZ_AMD_ERR_INVALID_ARG;  // slabs were not compressed with one shared codebook
    // every slab but the last must end on a chunk boundary, or the merged chunking differs
    if (p.ph.sublen <= 0) return PSZ_AMD_ERR_BAD_ARCHIVE;
    if (i + 1 < nparts && p.n % (size_t)p.ph.sublen != 0) return PSZ_ABORT_UNSUPPORTED_DIMENSION;
    // slabs split the slowest axis of the field: the faster extents must be the field's, and
    // every slab but the last must end on a prediction-tile boundary (z: 8 planes, 2-D: 32 rows,
    // 1-D: 1024 elements; launch.hh:47-121), or Lorenzo would cross the seam differently
    if (!slab_shape_ok(p.h.len, full_len, i + 1 == nparts)) return PSZ_ABORT_UNSUPPORTED_DIMENSION;
    if (elem_offsets && elem_offsets[i] != n_total) return PSZ_AMD_ERR_INVALID_ARG;  // slabs in field order
    n_total += p.n;
    splen += p.h.splen;
    ncell += p.ph.total_ncell;
    nbit += p.ph.total_nbit;
    pardeg += (size_t)p.ph.pardeg;
  }
  if (n_total != full_len.x * full_len.y * full_len.z || ncell >= (1ull << 32) || n_total >= (1ull << 32))
    return PSZ_ABORT_UNSUPPORTED_DIMENSION;

  const int bklen = P[0].ph.bklen;
  const size_t rv = rvbk_bytes(bklen);
  phf_header ph;
  std::memset(&ph, 0, sizeof(ph));
  ph.bklen = bklen, ph.sublen = P[0].ph.sublen, ph.pardeg = (int)pardeg, ph.original_len = n_total;
  ph.total_nbit = nbit, ph.total_ncell = ncell;
  ph.entry[PHFHEADER_HEADER] = 0;
  ph.entry[PHFHEADER_RVBK] = PHFHEADER_FORCED_ALIGN;
  ph.entry[PHFHEADER_PAR_NBIT] = (uint32_t)(PHFHEADER_FORCED_ALIGN + rv);
  ph.entry[PHFHEADER_PAR_ENTRY] = (uint32_t)(ph.entry[PHFHEADER_PAR_NBIT] + 4 * pardeg);
  ph.entry[PHFHEADER_BITSTREAM] = (uint32_t)(ph.entry[PHFHEADER_PAR_ENTRY] + 4 * pardeg);
  ph.entry[PHFHEADER_END] = (uint32_t)(ph.entry[PHFHEADER_BITSTREAM] + 4 * ncell);

  psz_header h = P[0].h;
  h.len = full_len;
  h.splen = splen;
  h.vle_sublen = ph.sublen, h.vle_pardeg = (int)pardeg;
  h.entry[PSZHEADER_HEADER] = 0;
  h.entry[PSZHEADER_ANCHOR] = sizeof(psz_header);
  h.entry[PSZHEADER_ENCODED] = sizeof(psz_header);
  h.entry[PSZHEADER_SPFMT] = h.entry[PSZHEADER_ENCODED] + ph.entry[PHFHEADER_END];
  h.entry[PSZHEADER_ENC_PASS1_END] = (uint32_t)(h.entry[PSZHEADER_SPFMT] + 8 * splen);
  h.entry[PSZHEADER_ENC_PASS2_END] = h.entry[PSZHEADER_ENC_PASS1_END];
  // extrema (Rel mode): the whole field's range
  for (const Part& p : P) {
    if (p.h.min_val < h.min_val) h.min_val = p.h.min_val;
    if (p.h.max_val > h.max_val) h.max_val = p.h.max_val;
  }
  const size_t total = h.entry[PSZHEADER_ENC_PASS2_END];
  *out_bytes = total;
  if (!out) return PSZ_SUCCESS;  // size query
  if (out_cap < total) return PSZ_AMD_ERR_INVALID_ARG;

  uint8_t* phf = out + h.entry[PSZHEADER_ENCODED];
  std::memcpy(out, &h, sizeof(h));
  std::memset(phf, 0, PHFHEADER_FORCED_ALIGN);
  std::memcpy(phf, &ph, sizeof(ph));
  std::memcpy(phf + PHFHEADER_FORCED_ALIGN, P[0].phf + PHFHEADER_FORCED_ALIGN, rv);
  uint32_t* nbit_out = reinterpret_cast<uint32_t*>(phf + ph.entry[PHFHEADER_PAR_NBIT]);
  uint32_t* entry_out = reinterpret_cast<uint32_t*>(phf + ph.entry[PHFHEADER_PAR_ENTRY]);
  uint8_t* bits_out = phf + ph.entry[PHFHEADER_BITSTREAM];
  uint8_t* cells_out = out + h.entry[PSZHEADER_SPFMT];
  size_t cell_base = 0, chunk_base = 0, ol_base = 0, elem_base = 0;
  for (const Part& p : P) {
    const size_t pd = (size_t)p.ph.pardeg, nc = p.ph.total_ncell;
    std::memcpy(nbit_out + chunk_base, p.phf + p.ph.entry[PHFHEADER_PAR_NBIT], 4 * pd);
    const uint32_t* ent = reinterpret_cast<const uint32_t*>(p.phf + p.ph.entry[PHFHEADER_PAR_ENTRY]);
    for (size_t c = 0; c < pd; c++) entry_out[chunk_base + c] = ent[c] + (uint32_t)cell_base;
    std::memcpy(bits_out + 4 * cell_base, p.phf + p.ph.entry[PHFHEADER_BITSTREAM], 4 * nc);
    const uint8_t* cells = p.base + p.h.entry[PSZHEADER_SPFMT];
    for (size_t k = 0; k < p.h.splen; k++) {
      uint32_t v[2];
      std::memcpy(v, cells + 8 * k, 8);
      v[1] += (uint32_t)elem_base;  // {f32 value, u32 index} (sp_interface.h:20-26)
      std::memcpy(cells_out + 8 * (ol_base + k), v, 8);
    }
    cell_base += nc, chunk_base += pd, ol_base += p.h.splen, elem_base += p.n;
  }
  return PSZ_SUCCESS;
}
