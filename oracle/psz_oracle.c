/* oracle/psz_oracle.c -- TEST INFRASTRUCTURE ONLY (see psz_oracle.h).
 *
 * Plain-C restatement of the reference GPU semantics.  It is the checker for the
 * HIP product path: tests compare cusz_amd's device results against it, and it is
 * itself pinned against the reference's own KATs (test/src/detail/correctness.inl)
 * and against the compiled reference CPU path (oracle/_ref, see tests/).
 *
 * Build with -ffp-contract=off: every floating-point operation below is a single
 * IEEE operation in the element type T, in the reference's order.
 */
#include "psz_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

int orc_ndim(size_t x, size_t y, size_t z)
{ /* psz/include/kernel/launch.hh:19-28 */
  if (z == 1 && y == 1) return 1;
  if (z == 1) return 2;
  return 3;
}

static inline uint16_t zz_enc(int16_t v)
{ /* psz/include/detail/composite.hh:61-70 */
  return (uint16_t)(((uint16_t)v << 1) ^ (uint16_t)(v >> 15));
}
static inline int16_t zz_dec(uint16_t u)
{ /* psz/include/detail/composite.hh:72-83 */
  return (int16_t)((u >> 1) ^ (uint16_t)(-(int16_t)(u & 1)));
}

/* ------------------------------------------------------------------------- */
/* Lorenzo predict-quantize.  T = element type, R = round function.            */
/* ------------------------------------------------------------------------- */

#define DEFINE_LRZ_C(NAME, T, ROUND, FABS)                                                     \
  size_t NAME(const T* in, size_t lx, size_t ly, size_t lz, double eb, uint16_t radius,        \
              int zigzag, uint16_t* codes, float* ol_val, uint32_t* ol_idx, size_t ol_cap)     \
  {                                                                                            \
    /* lrz_c.cuhip.inl:489: ebx2_r = 1/(2eb) in double, passed as (T) */                       \
    const T ebx2_r = (T)(1.0 / (eb * 2));                                                      \
    const T r = (T)radius;                                                                     \
    size_t nol = 0;                                                                            \
    /* collect outliers in (tile-order) then sort by index at the end */                       \
    size_t n = lx * ly * lz;                                                                   \
    int d = orc_ndim(lx, ly, lz);                                                              \
    uint8_t* isol = (uint8_t*)calloc(n ? n : 1, 1);                                            \
    float* olv_dense = (float*)malloc(sizeof(float) * (n ? n : 1));                            \
    if (d == 1) {                                                                              \
      /* lrz_c.cuhip.inl:23-109: tile 1024 */                                                  \
      const size_t TD = 1024;                                                                  \
      T p[1024];                                                                               \
      for (size_t base = 0; base < n; base += TD) {                                            \
        for (size_t i = 0; i < TD; i++) {                                                      \
          size_t id = base + i;                                                                \
          p[i] = id < n ? ROUND(in[id] * ebx2_r) : (T)0;                                       \
        }                                                                                      \
        for (size_t i = 0; i < TD && base + i < n; i++) {                                      \
          T delta = p[i] - (i > 0 ? p[i - 1] : (T)0);                                          \
          LRZ_QUANT(T, FABS, delta, base + i);                                                 \
        }                                                                                      \
      }                                                                                        \
    }                                                                                          \
    else if (d == 2) {                                                                         \
      /* lrz_c.cuhip.inl:187-273: tile 32x32; y-diff then x-diff of y-diffs */                 \
      const size_t TD = 32;                                                                    \
      T p[33][32], a[32][32];                                                                  \
      for (size_t by = 0; by < ly; by += TD)                                                   \
        for (size_t bx = 0; bx < lx; bx += TD) {                                               \
          for (size_t x = 0; x < TD; x++) p[0][x] = (T)0;                                      \
          for (size_t y = 0; y < TD; y++)                                                      \
            for (size_t x = 0; x < TD; x++) {                                                  \
              size_t gx = bx + x, gy = by + y;                                                 \
              p[y + 1][x] = (gx < lx && gy < ly) ? ROUND(in[gy * lx + gx] * ebx2_r) : (T)0;    \
            }                                                                                  \
          for (size_t y = 0; y < TD; y++)                                                      \
            for (size_t x = 0; x < TD; x++) a[y][x] = p[y + 1][x] - p[y][x];                   \
          for (size_t y = 0; y < TD; y++)                                                      \
            for (size_t x = 0; x < TD; x++) {                                                  \
              size_t gx = bx + x, gy = by + y;                                                 \
              if (!(gx < lx && gy < ly)) continue;                                             \
              T delta = x > 0 ? a[y][x] - a[y][x - 1] : a[y][x];                               \
              LRZ_QUANT(T, FABS, delta, gy * lx + gx);                                         \
            }                                                                                  \
        }                                                                                      \
    }                                                                                          \
    else {                                                                                     \
      /* lrz_c.cuhip.inl:275-372: tile 8^3; z-diff, then x-diff, then y-diff */                \
      const size_t TD = 8;                                                                     \
      T p[9][8][8], a[8][8][8], b[8][8][8];                                                    \
      for (size_t bz = 0; bz < lz; bz += TD)                                                   \
        for (size_t by = 0; by < ly; by += TD)                                                 \
          for (size_t bx = 0; bx < lx; bx += TD) {                                             \
            for (size_t y = 0; y < TD; y++)                                                    \
              for (size_t x = 0; x < TD; x++) p[0][y][x] = (T)0;                               \
            for (size_t z = 0; z < TD; z++)                                                    \
              for (size_t y = 0; y < TD; y++)                                                  \
                for (size_t x = 0; x < TD; x++) {                                              \
                  size_t gx = bx + x, gy = by + y, gz = bz + z;                                \
                  p[z + 1][y][x] = (gx < lx && gy < ly && gz < lz)                             \
                                       ? ROUND(in[(gz * ly + gy) * lx + gx] * ebx2_r)          \
                                       : (T)0;                                                 \
                }                                                                              \
            for (size_t z = 0; z < TD; z++)                                                    \
              for (size_t y = 0; y < TD; y++)                                                  \
                for (size_t x = 0; x < TD; x++) a[z][y][x] = p[z + 1][y][x] - p[z][y][x];      \
            for (size_t z = 0; z < TD; z++)                                                    \
              for (size_t y = 0; y < TD; y++)                                                  \
                for (size_t x = 0; x < TD; x++)                                                \
                  b[z][y][x] = x > 0 ? a[z][y][x] - a[z][y][x - 1] : a[z][y][x];               \
            for (size_t z = 0; z < TD; z++)                                                    \
              for (size_t y = 0; y < TD; y++)                                                  \
                for (size_t x = 0; x < TD; x++) {                                              \
                  size_t gx = bx + x, gy = by + y, gz = bz + z;                                \
                  if (!(gx < lx && gy < ly && gz < lz)) continue;                              \
                  /* (threadIdx.y > 0) * s[y][x]: row y=0 subtracts 0 */                       \
                  T delta = y > 0 ? b[z][y][x] - b[z][y - 1][x] : b[z][y][x];                  \
                  LRZ_QUANT(T, FABS, delta, (gz * ly + gy) * lx + gx);                         \
                }                                                                              \
          }                                                                                    \
    }                                                                                          \
    for (size_t i = 0; i < n; i++)                                                             \
      if (isol[i]) {                                                                           \
        if (nol < ol_cap) {                                                                    \
          ol_val[nol] = olv_dense[i];                                                          \
          ol_idx[nol] = (uint32_t)i;                                                           \
        }                                                                                      \
        nol++;                                                                                 \
      }                                                                                        \
    free(isol);                                                                                \
    free(olv_dense);                                                                           \
    return nol;                                                                                \
  }

/* quantize (lrz_c.cuhip.inl:310-331, composite.hh:61-70) */
#define LRZ_QUANT(T, FABS, DELTA, GID)                                       \
  do {                                                                       \
    T _delta = (DELTA);                                                      \
    int _q = FABS(_delta) < r;                                               \
    T _cand;                                                                 \
    if (zigzag) {                                                            \
      _cand = _delta;                                                        \
      codes[(GID)] = _q ? zz_enc((int16_t)_delta) : (uint16_t)0;             \
    }                                                                        \
    else {                                                                   \
      _cand = _delta + r;                                                    \
      codes[(GID)] = _q ? (uint16_t)_cand : (uint16_t)0;                     \
    }                                                                        \
    if (!_q) {                                                               \
      isol[(GID)] = 1;                                                       \
      olv_dense[(GID)] = (float)_cand;                                       \
    }                                                                        \
  } while (0)

DEFINE_LRZ_C(orc_lorenzo_c_f32, float, roundf, fabsf)
DEFINE_LRZ_C(orc_lorenzo_c_f64, double, round, fabs)

/* ------------------------------------------------------------------------- */
/* Lorenzo reconstruct, exact reference scan order.                           */
/* ------------------------------------------------------------------------- */

#define DEFINE_LRZ_X(NAME, T)                                                                   \
  void NAME(const uint16_t* codes, const float* ol_val, const uint32_t* ol_idx, size_t nol,     \
            size_t lx, size_t ly, size_t lz, double eb, uint16_t radius, int zigzag, T* out)    \
  {                                                                                             \
    const T ebx2 = (T)(eb * 2); /* lrz_x.cuhip.inl:432 */                                       \
    const T r = (T)radius;                                                                      \
    size_t n = lx * ly * lz;                                                                    \
    int d = orc_ndim(lx, ly, lz);                                                               \
    /* scatter onto a zero plane: spvn.cuhip.inl:41-50 */                                       \
    T* plane = (T*)calloc(n ? n : 1, sizeof(T));                                                \
    for (size_t i = 0; i < nol; i++)                                                            \
      if (ol_idx[i] < n) plane[ol_idx[i]] = (T)ol_val[i];                                       \
    /* fused value (lrz_x.cuhip.inl:37,202,301) */                                              \
    if (d == 1) {                                                                               \
      /* lrz_x.cuhip.inl:11-78 + wave32.cuhip.inl:7-66; 256 threads x 4 */                      \
      T v[1024];                                                                                \
      for (size_t base = 0; base < n; base += 1024) {                                           \
        for (size_t i = 0; i < 1024; i++) {                                                     \
          size_t id = base + i;                                                                 \
          v[i] = id < n ? LRZ_FUSE(T, id) : (T)0;                                               \
        }                                                                                       \
        T addend[256], tmp[256];                                                                \
        for (int t = 0; t < 256; t++) {                                                         \
          for (int i = 1; i < 4; i++) v[t * 4 + i] += v[t * 4 + i - 1];                         \
          addend[t] = v[t * 4 + 3];                                                             \
        }                                                                                       \
        for (int dd = 1; dd < 32; dd *= 2) {                                                    \
          memcpy(tmp, addend, sizeof(tmp));                                                     \
          for (int t = 0; t < 256; t++)                                                         \
            if (t % 32 >= dd) addend[t] = tmp[t] + tmp[t - dd];                                 \
        }                                                                                       \
        for (int t = 0; t < 256; t++)                                                           \
          if (t % 32 > 0)                                                                       \
            for (int i = 0; i < 4; i++) v[t * 4 + i] += addend[t - 1];                          \
        T ex_in[8], ex_out[8];                                                                  \
        for (int w = 0; w < 8; w++) ex_in[w] = v[(w * 32 + 31) * 4 + 3];                        \
        ex_out[0] = 0;                                                                          \
        for (int w = 1; w < 8; w++) ex_out[w] = ex_out[w - 1] + ex_in[w - 1];                   \
        for (int t = 0; t < 256; t++)                                                           \
          for (int i = 0; i < 4; i++) v[t * 4 + i] += ex_out[t / 32];                           \
        for (size_t i = 0; i < 1024 && base + i < n; i++) out[base + i] = v[i] * ebx2;          \
      }                                                                                         \
    }                                                                                           \
    else if (d == 2) {                                                                          \
      /* lrz_x.cuhip.inl:178-269; tile 32x32, 4 strips of 8 rows */                             \
      T v[32][32], tmp[32];                                                                     \
      for (size_t by = 0; by < ly; by += 32)                                                    \
        for (size_t bx = 0; bx < lx; bx += 32) {                                                \
          for (size_t y = 0; y < 32; y++)                                                       \
            for (size_t x = 0; x < 32; x++) {                                                   \
              size_t gx = bx + x, gy = by + y, id = gy * lx + gx;                               \
              v[y][x] = (gx < lx && gy < ly) ? LRZ_FUSE(T, id) : (T)0;                          \
            }                                                                                   \
          for (int s = 0; s < 4; s++)                                                           \
            for (int i = 1; i < 8; i++)                                                         \
              for (int x = 0; x < 32; x++) v[s * 8 + i][x] += v[s * 8 + i - 1][x];              \
          for (int x = 0; x < 32; x++) {                                                        \
            T s0 = v[7][x], s1 = v[15][x], s2 = v[23][x];                                       \
            T acc1 = s1 + s0;                                                                   \
            T acc2 = s2 + acc1;                                                                 \
            for (int i = 0; i < 8; i++) {                                                       \
              v[8 + i][x] += s0;                                                                \
              v[16 + i][x] += acc1;                                                             \
              v[24 + i][x] += acc2;                                                             \
            }                                                                                   \
          }                                                                                     \
          for (int y = 0; y < 32; y++)                                                          \
            for (int dd = 1; dd < 32; dd *= 2) {                                                \
              memcpy(tmp, v[y], sizeof(tmp));                                                   \
              for (int x = dd; x < 32; x++) v[y][x] = tmp[x] + tmp[x - dd];                     \
            }                                                                                   \
          for (size_t y = 0; y < 32; y++)                                                       \
            for (size_t x = 0; x < 32; x++) {                                                   \
              size_t gx = bx + x, gy = by + y;                                                  \
              if (gx < lx && gy < ly) out[gy * lx + gx] = v[y][x] * ebx2;                       \
            }                                                                                   \
        }                                                                                       \
    }                                                                                           \
    else {                                                                                      \
      /* lrz_x.cuhip.inl:271-360; y sequential, x then z Hillis-Steele (width 8) */             \
      T v[8][8][8], tmp[8];                                                                     \
      for (size_t bz = 0; bz < lz; bz += 8)                                                     \
        for (size_t by = 0; by < ly; by += 8)                                                   \
          for (size_t bx = 0; bx < lx; bx += 8) {                                               \
            for (size_t z = 0; z < 8; z++)                                                      \
              for (size_t y = 0; y < 8; y++)                                                    \
                for (size_t x = 0; x < 8; x++) {                                                \
                  size_t gx = bx + x, gy = by + y, gz = bz + z, id = (gz * ly + gy) * lx + gx;  \
                  v[z][y][x] = (gx < lx && gy < ly && gz < lz) ? LRZ_FUSE(T, id) : (T)0;        \
                }                                                                               \
            for (int z = 0; z < 8; z++)                                                         \
              for (int y = 1; y < 8; y++)                                                       \
                for (int x = 0; x < 8; x++) v[z][y][x] += v[z][y - 1][x];                       \
            for (int z = 0; z < 8; z++)                                                         \
              for (int y = 0; y < 8; y++)                                                       \
                for (int dd = 1; dd < 8; dd *= 2) {                                             \
                  memcpy(tmp, v[z][y], sizeof(tmp));                                            \
                  for (int x = dd; x < 8; x++) v[z][y][x] = tmp[x] + tmp[x - dd];               \
                }                                                                               \
            for (int y = 0; y < 8; y++)                                                         \
              for (int x = 0; x < 8; x++)                                                       \
                for (int dd = 1; dd < 8; dd *= 2) {                                             \
                  for (int z = 0; z < 8; z++) tmp[z] = v[z][y][x];                              \
                  for (int z = dd; z < 8; z++) v[z][y][x] = tmp[z] + tmp[z - dd];               \
                }                                                                               \
            for (size_t z = 0; z < 8; z++)                                                      \
              for (size_t y = 0; y < 8; y++)                                                    \
                for (size_t x = 0; x < 8; x++) {                                                \
                  size_t gx = bx + x, gy = by + y, gz = bz + z;                                 \
                  if (gx < lx && gy < ly && gz < lz)                                            \
                    out[(gz * ly + gy) * lx + gx] = v[z][y][x] * ebx2;                          \
                }                                                                               \
          }                                                                                     \
    }                                                                                           \
    free(plane);                                                                                \
  }

#define LRZ_FUSE(T, ID) \
  (zigzag ? plane[(ID)] + (T)zz_dec(codes[(ID)]) : plane[(ID)] + (T)codes[(ID)] - r)

DEFINE_LRZ_X(orc_lorenzo_x_f32, float)
DEFINE_LRZ_X(orc_lorenzo_x_f64, double)

/* ------------------------------------------------------------------------- */
/* histogram                                                                  */
/* ------------------------------------------------------------------------- */

void orc_histogram_u2(const uint16_t* codes, size_t n, uint32_t* hist, int bklen)
{
  memset(hist, 0, sizeof(uint32_t) * bklen);
  for (size_t i = 0; i < n; i++)
    if (codes[i] < bklen) hist[codes[i]]++;
}

/* ------------------------------------------------------------------------- */
/* Huffman code lengths: the reference's binary heap (hf_bk_impl1.seq.cc)      */
/* ------------------------------------------------------------------------- */

typedef struct {
  int left, right; /* -1 for leaves */
  uint64_t freq;
  int sym;
} orc_node;

typedef struct {
  orc_node* pool;
  int npool;
  int* qq; /* 1-based heap of node ids */
  int qend;
} orc_heap;

/* qinsert, hf_bk_impl1.seq.cc:103-112 */
static void heap_insert(orc_heap* h, int n)
{
  int j, i = h->qend++;
  while ((j = (i >> 1))) {
    if (h->pool[h->qq[j]].freq <= h->pool[n].freq) break;
    h->qq[i] = h->qq[j], i = j;
  }
  h->qq[i] = n;
}

/* qremove, hf_bk_impl1.seq.cc:114-137 */
static int heap_remove(orc_heap* h)
{
  int i, l;
  int n = h->qq[i = 1];
  if (h->qend < 2) return -1;
  h->qend--;
  h->qq[i] = h->qq[h->qend];
  while ((l = (i << 1)) < h->qend) {
    if (l + 1 < h->qend && h->pool[h->qq[l + 1]].freq < h->pool[h->qq[l]].freq) l++;
    if (h->pool[h->qq[i]].freq > h->pool[h->qq[l]].freq) {
      int p = h->qq[i];
      h->qq[i] = h->qq[l];
      h->qq[l] = p;
      i = l;
    }
    else
      break;
  }
  return n;
}

#define ORC_LMAX 27

/* deterministic length limit (deviation from the reference's broken 28-bit code,
 * hf_bk.seq.cc:108-112; see DESIGN.md "Codebook") */
static void limit_lengths(const uint32_t* hist, int bklen, uint8_t* lens)
{
  const uint64_t cap = 1ull << ORC_LMAX;
  uint64_t K = 0;
  for (int i = 0; i < bklen; i++)
    if (lens[i]) {
      if (lens[i] > ORC_LMAX) lens[i] = ORC_LMAX;
      K += 1ull << (ORC_LMAX - lens[i]);
    }
  while (K > cap) {
    int best = -1;
    for (int i = 0; i < bklen; i++) {
      if (!lens[i] || lens[i] >= ORC_LMAX) continue;
      if (best < 0 || lens[i] > lens[best] ||
          (lens[i] == lens[best] && (hist[i] < hist[best] || (hist[i] == hist[best] && i > best))))
        best = i;
    }
    K -= 1ull << (ORC_LMAX - lens[best] - 1);
    lens[best]++;
  }
}

int orc_huffman_lengths(const uint32_t* hist, int bklen, uint8_t* lens)
{
  memset(lens, 0, bklen);
  int nused = 0, last = -1;
  for (int i = 0; i < bklen; i++)
    if (hist[i]) nused++, last = i;
  if (nused == 0) return 0;
  if (nused == 1) { /* deviation: 1-bit code instead of the reference's 0-bit code */
    lens[last] = 1;
    return 1;
  }
  orc_heap h;
  h.pool = (orc_node*)calloc(2 * bklen + 2, sizeof(orc_node));
  h.qq = (int*)calloc(2 * bklen + 4, sizeof(int));
  h.npool = 0;
  h.qend = 1;
  /* leaves in symbol order: hf_bk_impl1.seq.cc:192-193 */
  for (int i = 0; i < bklen; i++)
    if (hist[i]) {
      orc_node* nd = &h.pool[h.npool];
      nd->left = nd->right = -1, nd->freq = hist[i], nd->sym = i;
      heap_insert(&h, h.npool++);
    }
  /* merges: hf_bk_impl1.seq.cc:194 */
  while (h.qend > 2) {
    int a = heap_remove(&h);
    int b = heap_remove(&h);
    orc_node* nd = &h.pool[h.npool];
    nd->left = a, nd->right = b, nd->freq = h.pool[a].freq + h.pool[b].freq, nd->sym = -1;
    heap_insert(&h, h.npool++);
  }
  /* depths (in-order traversal, hf_bk_internal.seq.cc:64-107) */
  int root = h.qq[1];
  int* stack = (int*)malloc(sizeof(int) * (2 * bklen + 2));
  int* depth = (int*)malloc(sizeof(int) * (2 * bklen + 2));
  int sp = 0, maxl = 0;
  stack[sp] = root, depth[sp] = 0, sp++;
  while (sp) {
    sp--;
    int nd = stack[sp], dd = depth[sp];
    if (h.pool[nd].left < 0) {
      int l = dd > 255 ? 255 : dd;
      lens[h.pool[nd].sym] = (uint8_t)l;
      if (l > maxl) maxl = l;
    }
    else {
      stack[sp] = h.pool[nd].left, depth[sp] = dd + 1, sp++;
      stack[sp] = h.pool[nd].right, depth[sp] = dd + 1, sp++;
    }
  }
  free(stack);
  free(depth);
  free(h.pool);
  free(h.qq);
  if (maxl > ORC_LMAX) {
    limit_lengths(hist, bklen, lens);
    maxl = ORC_LMAX;
  }
  return maxl;
}

/* canonisation, hf_canon.seq.cc:105-161; book word = code | len<<27 (hf_impl.hh:40-59) */
static int canonize_lengths(uint8_t* lens, int bklen, uint32_t* book, uint8_t* revbook);

int orc_build_codebook_u2(const uint32_t* hist, int bklen, uint32_t* book, uint8_t* revbook)
{
  uint8_t* lens = (uint8_t*)malloc(bklen);
  orc_huffman_lengths(hist, bklen, lens);
  return canonize_lengths(lens, bklen, book, revbook);
}

/* ------------------------------------------------------------------------- */
/* Device codebook (cusz_amd/csrc/book_device.hh) restated serially: NOT the reference's heap.  */
/* Optimal code lengths by the two-queue Huffman construction: leaves sorted by (weight, symbol), */
/* internal nodes in creation order (their weights never decrease), at each merge the two       */
/* smallest heads with a leaf taken before an internal node of equal weight.  Weights are       */
/* hist + smooth (smooth = 1: every symbol encodable, the sampled-codebook mode); a tree deeper  */
/* than 27 bits halves every weight ((w + 1) / 2, never 0) and is rebuilt.  Canonisation as the  */
/* reference's (canonize_lengths).  Test infrastructure: the device book is checked against it. */
/* ------------------------------------------------------------------------- */

static int twoqueue_lengths(const uint64_t* w, int bklen, uint8_t* lens)
{
  int n = 0;
  int* sym = (int*)malloc(sizeof(int) * bklen);
  for (int s = 0; s < bklen; s++)
    if (w[s]) sym[n++] = s;
  memset(lens, 0, bklen);
  if (n == 0) {
    free(sym);
    return 0;
  }
  if (n == 1) {
    lens[sym[0]] = 1;
    free(sym);
    return 1;
  }
  /* stable sort of the used symbols by weight (insertion sort: ties keep symbol order) */
  for (int i = 1; i < n; i++) {
    int v = sym[i], j = i - 1;
    while (j >= 0 && w[sym[j]] > w[v]) sym[j + 1] = sym[j], j--;
    sym[j + 1] = v;
  }
  uint64_t* iw = (uint64_t*)malloc(sizeof(uint64_t) * n);
  int* par = (int*)malloc(sizeof(int) * 2 * n);  /* leaves 0..n-1 (sorted order), internals n.. */
  int li = 0, ii = 0, ni = 0;
  while ((n - li) + (ni - ii) > 1) {
    int pick[2];
    uint64_t pw[2];
    for (int k = 0; k < 2; k++) {
      const int hasl = li < n, hasi = ii < ni;
      if (hasl && (!hasi || w[sym[li]] <= iw[ii])) pick[k] = li, pw[k] = w[sym[li]], li++;
      else pick[k] = n + ii, pw[k] = iw[ii], ii++;
    }
    par[pick[0]] = par[pick[1]] = n + ni;
    iw[ni++] = pw[0] + pw[1];
  }
  /* depths: the root is the last internal node; parents come after their children */
  int* depth = (int*)malloc(sizeof(int) * 2 * n);
  const int root = n + ni - 1;
  int maxl = 0;
  depth[root] = 0;
  for (int id = root - 1; id >= 0; id--) {
    depth[id] = depth[par[id]] + 1;
    if (id < n) {
      lens[sym[id]] = (uint8_t)(depth[id] > 255 ? 255 : depth[id]);
      if (depth[id] > maxl) maxl = depth[id];
    }
  }
  free(depth);
  free(par);
  free(iw);
  free(sym);
  return maxl;
}

int orc_book_twoqueue_u2(const uint32_t* hist, int bklen, uint32_t smooth, uint32_t* book, uint8_t* revbook)
{
  uint64_t* w = (uint64_t*)malloc(sizeof(uint64_t) * bklen);
  uint8_t* lens = (uint8_t*)malloc(bklen);
  for (int s = 0; s < bklen; s++) w[s] = (uint64_t)hist[s] + smooth;
  while (twoqueue_lengths(w, bklen, lens) > ORC_LMAX)
    for (int s = 0; s < bklen; s++)
      if (w[s]) w[s] = (w[s] + 1) / 2;
  free(w);
  return canonize_lengths(lens, bklen, book, revbook);
}

/* lens: consumed (freed) */
static int canonize_lengths(uint8_t* lens, int bklen, uint32_t* book, uint8_t* revbook)
{
  const int TB = 32;
  int rvbk_bytes = 4 * (2 * TB) + 2 * bklen;

  int numl[32] = {0}, iterby[32] = {0}, first[32] = {0}, entry[32] = {0};
  uint16_t* keys = (uint16_t*)calloc(bklen, sizeof(uint16_t));
  uint32_t* canon = (uint32_t*)malloc(sizeof(uint32_t) * bklen);
  int max_l = 0;
  for (int i = 0; i < bklen; i++)
    if (lens[i]) {
      if (lens[i] > max_l) max_l = lens[i];
      numl[lens[i]]++;
    }
  for (int i = 1; i < TB; i++) entry[i] = numl[i - 1];
  for (int i = 1; i < TB; i++) entry[i] += entry[i - 1];
  for (int i = 0; i < TB; i++) iterby[i] = entry[i];
  first[max_l] = 0;
  for (int l = max_l - 1; l >= 1; l--) first[l] = (first[l + 1] + numl[l + 1] + 1) / 2;
  first[0] = 0xff;
  for (int i = 0; i < bklen; i++) canon[i] = 0xFFFFFFFFu, book[i] = 0xFFFFFFFFu;
  for (int i = 0; i < bklen; i++) {
    int l = lens[i];
    if (l) {
      canon[iterby[l]] = ((uint32_t)(first[l] + iterby[l] - entry[l]) & 0x07FFFFFFu) |
                         ((uint32_t)l << 27);
      keys[iterby[l]] = (uint16_t)i;
      iterby[l]++;
    }
  }
  for (int i = 0; i < bklen; i++)
    if (canon[i] != 0xFFFFFFFFu) book[keys[i]] = canon[i];

  memset(revbook, 0, rvbk_bytes);
  memcpy(revbook, first, 4 * TB);
  memcpy(revbook + 4 * TB, entry, 4 * TB);
  memcpy(revbook + 8 * TB, keys, 2 * bklen);
  free(lens);
  free(keys);
  free(canon);
  return rvbk_bytes;
}

/* ------------------------------------------------------------------------- */
/* coarse-grained Huffman encode/decode                                       */
/* ------------------------------------------------------------------------- */

void orc_coarse_tune(size_t len, int n_cu, int max_threads, int* sublen, int* pardeg)
{ /* libphf.cc:26-70 (PHF_DEFLATE_CONSTANT 4, BLOCK_DIM_DEFLATE 256) */
  size_t nthread = (size_t)max_threads * (size_t)n_cu / 4;
  size_t s = (len - 1) / nthread + 1;
  s = ((s - 1) / 256 + 1) * 256;
  *sublen = (int)s;
  *pardeg = (int)((len - 1) / s + 1);
}

size_t orc_hf_encode_u2(const uint16_t* codes, size_t n, const uint32_t* book, int sublen,
                        uint32_t* par_nbit, uint32_t* par_entry, uint32_t* bitstream,
                        size_t bitstream_cap, uint64_t* total_nbit)
{
  size_t pardeg = (n - 1) / sublen + 1;
  size_t cell = 0;
  uint64_t tb = 0;
  for (size_t c = 0; c < pardeg; c++) {
    size_t s = c * sublen, e = s + sublen < n ? s + sublen : n;
    uint32_t nbit = 0, buf = 0;
    int fill = 0; /* bits used in buf */
    par_entry[c] = (uint32_t)cell;
    for (size_t i = s; i < e; i++) {
      uint32_t w = book[codes[i]];
      int len = (int)(w >> 27);
      uint32_t code = w & 0x07FFFFFFu;
      nbit += len;
      /* MSB-first append (hf_kernels.cuhip.inl:114-151) */
      while (len > 0) {
        int room = 32 - fill;
        int take = len < room ? len : room;
        uint32_t part = (code >> (len - take)) & (take == 32 ? 0xFFFFFFFFu : ((1u << take) - 1));
        buf |= part << (room - take);
        fill += take;
        len -= take;
        if (fill == 32) {
          if (cell >= bitstream_cap) return (size_t)-1;
          bitstream[cell++] = buf;
          buf = 0, fill = 0;
        }
      }
    }
    if (fill) {
      if (cell >= bitstream_cap) return (size_t)-1;
      bitstream[cell++] = buf;
    }
    par_nbit[c] = nbit;
    tb += nbit;
  }
  if (total_nbit) *total_nbit = tb;
  return cell;
}

void orc_hf_decode_u2(const uint32_t* bitstream, const uint8_t* revbook, int bklen,
                      const uint32_t* par_nbit, const uint32_t* par_entry, int sublen,
                      int pardeg, size_t n, uint16_t* out)
{ /* hf_kernels.cuhip.inl:341-380 */
  const uint32_t* first = (const uint32_t*)revbook;
  const uint32_t* entry = first + 32;
  const uint16_t* keys = (const uint16_t*)(revbook + 4 * 64);
  (void)bklen;
  for (int g = 0; g < pardeg; g++) {
    const uint32_t* in = bitstream + par_entry[g];
    uint32_t total_bw = par_nbit[g];
    uint32_t ncell = (total_bw + 31) / 32;
    size_t ob = (size_t)g * sublen, oe = ob + sublen < n ? ob + sublen : n;
#define RD(k) ((k) < ncell ? in[(k)] : 0u)
    uint32_t i = 0, idx_bit, idx_byte;
    uint32_t bufr = RD(0);
    uint32_t v = (bufr >> 31) & 1;
    int l = 1;
    size_t o = ob;
    while (i < total_bw) {
      while (v < first[l]) {
        ++i;
        idx_byte = i / 32, idx_bit = i % 32;
        if (idx_bit == 0) bufr = RD(idx_byte);
        v = (v << 1) | ((bufr >> (31 - idx_bit)) & 1);
        ++l;
      }
      if (o < oe) out[o] = keys[entry[l] + v - first[l]];
      o++;
      ++i;
      idx_byte = i / 32, idx_bit = i % 32;
      if (idx_bit == 0) bufr = RD(idx_byte);
      v = (bufr >> (31 - idx_bit)) & 1;
      l = 1;
    }
#undef RD
  }
}
