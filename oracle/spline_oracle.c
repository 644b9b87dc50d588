/* oracle/spline_oracle.c -- TEST INFRASTRUCTURE ONLY (see psz_oracle.h).
 *
 * CPU restatement of cuSZ-i's spline3 predictor-quantizer and its reconstruction,
 * psz/src/kernel/detail/spline3.inl (kernels at :916-1016, interpolation schedule at
 * :678-900, per-point rule at :391-618) launched by psz/src/kernel/spline3.cu:22-63.
 *
 * PARITY UNPINNED: the reference has no test, fixture or working pipeline for this path
 * (compressor.inl:358-361 and :495-497 call a null stub), so this file is pinned only by
 * reading the source; tests check the GPU against it bit for bit and check properties
 * (error bound, anchor exactness, code round trip).
 *
 * Tile = 32 x 8 x 8 data points, processed on a 33 x 9 x 9 scratch that includes the +1
 * faces of the next tiles (spline3.cu:29: grid = ceil(x/32), ceil(y/8), ceil(z/8)).  Each
 * tile is self-contained: faces shared with a neighbour are recomputed identically there.
 * Outlier order (the reference's is an atomicAdd race, spline3.inl:386-396): tile order
 * (x fastest over tiles), then the tile's points in (z, y, x) order -- the deterministic
 * order the GPU build writes.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "psz_oracle.h"

#define SX 33
#define SY 9
#define SZ 9
#define SIDX(x, y, z) ((x) + SX * ((y) + SY * (z)))

typedef struct {
  unsigned bx, by, bz, gdx, gdy, gdz; /* tile index and grid (BIX.., GDX..) */
  size_t X, Y, Z;                     /* data_size */
} tile_ctx;

/* xyz33x9x9_predicate (spline3.inl:145-157) */
static int pred_ok(const tile_ctx* t, int inclusive, int x, int y, int z)
{
  const size_t gx = (size_t)t->bx * 32 + x, gy = (size_t)t->by * 8 + y, gz = (size_t)t->bz * 8 + z;
  if (!(gx < t->X && gy < t->Y && gz < t->Z)) return 0;
  if (inclusive) return x <= 32 && y <= 8 && z <= 8;
  return x < 32 + (t->bx == t->gdx - 1) && y < 8 + (t->by == t->gdy - 1) && z < 8 + (t->bz == t->gdz - 1);
}

/* the per-point rule of interpolate_stage (spline3.inl:391-618), T = float and double.
 * DIR 0 = BLUE (along z), 1 = YELLOW (along y), 2 = HOLLOW (along x).  The operation order
 * of every expression is the reference's (left to right, no contraction). */
#define DEFINE_SPLINE(SUF, T, FABS)                                                              \
  static T SUF##_pred(const T* s, const tile_ctx* t, int dir, int x, int y, int z, int u)        \
  {                                                                                              \
    int c, blk, stride;                                                                          \
    size_t g, dsz;                                                                               \
    int last;                                                                                    \
    if (dir == 0) c = z, blk = 8, stride = SX * SY, g = (size_t)t->bz * 8 + z, dsz = t->Z, last = t->bz == t->gdz - 1; \
    else if (dir == 1) c = y, blk = 8, stride = SX, g = (size_t)t->by * 8 + y, dsz = t->Y, last = t->by == t->gdy - 1; \
    else c = x, blk = 32, stride = 1, g = (size_t)t->bx * 32 + x, dsz = t->X, last = t->bx == t->gdx - 1; \
    const int i = SIDX(x, y, z);                                                                 \
    const T* p = s + i;                                                                          \
    const int m3 = -3 * u * stride, m1 = -u * stride, p1 = u * stride, p3 = 3 * u * stride;      \
    if (!last) {                                                                                 \
      if (c >= 3 * u && c + 3 * u <= blk)                                                        \
        return (-p[m3] + 9 * p[m1] + 9 * p[p1] - p[p3]) / 16;                                    \
      else if (c + 3 * u <= blk)                                                                 \
        return (3 * p[m1] + 6 * p[p1] - p[p3]) / 8;                                              \
      else if (c >= 3 * u)                                                                       \
        return (-p[m3] + 6 * p[m1] + 3 * p[p1]) / 8;                                             \
      else                                                                                       \
        return (p[m1] + p[p1]) / 2;                                                              \
    }                                                                                            \
    if (c >= 3 * u) {                                                                            \
      if (c + 3 * u <= blk && g + 3 * u < dsz)                                                   \
        return (-p[m3] + 9 * p[m1] + 9 * p[p1] - p[p3]) / 16;                                    \
      else if (g + u < dsz)                                                                      \
        return (-p[m3] + 6 * p[m1] + 3 * p[p1]) / 8;                                             \
      else                                                                                       \
        return p[m1];                                                                            \
    }                                                                                            \
    if (c + 3 * u <= blk && g + 3 * u < dsz)                                                     \
      return (3 * p[m1] + 6 * p[p1] - p[p3]) / 8;                                                \
    else if (g + u < dsz)                                                                        \
      return (p[m1] + p[p1]) / 2;                                                                \
    else                                                                                         \
      return p[m1];                                                                              \
  }                                                                                              \
                                                                                                 \
  /* one stage: points (xm(ix), ym(iy), zm(iz)) for i < (DX, DY, DZ) (spline3.inl:620-660) */   \
  static void SUF##_stage(T* s, T* e, const tile_ctx* t, int dir, int u, int DX, int DY, int DZ, \
                          int incl, float eb_r, float ebx2, int radius, int compress)            \
  {                                                                                              \
    for (int iz = 0; iz < DZ; iz++)                                                              \
      for (int iy = 0; iy < DY; iy++)                                                            \
        for (int ix = 0; ix < DX; ix++) {                                                        \
          int x, y, z;                                                                           \
          if (dir == 0) x = u * (ix * 2), y = u * (iy * 2), z = u * (iz * 2 + 1);                \
          else if (dir == 1) x = u * (ix * 2), y = u * (iy * 2 + 1), z = u * iz;                 \
          else x = u * (ix * 2 + 1), y = u * iy, z = u * iz;                                     \
          if (!pred_ok(t, incl, x, y, z)) continue;                                              \
          const T pred = SUF##_pred(s, t, dir, x, y, z, u);                                      \
          const int i = SIDX(x, y, z);                                                           \
          if (compress) {                                                                        \
            const T err = s[i] - pred;                                                           \
            T code = FABS(err) * (T)eb_r + 1;                                                    \
            code = err < 0 ? -code : code;                                                       \
            code = (T)((int)(code / 2) + radius);                                                \
            e[i] = code;                                                                         \
            s[i] = pred + (code - radius) * (T)ebx2;                                             \
          } else {                                                                               \
            const T code = e[i];                                                                 \
            s[i] = pred + (code - radius) * (T)ebx2;                                             \
          }                                                                                      \
        }                                                                                        \
  }                                                                                              \
                                                                                                 \
  /* spline3d_layout2_interpolate, reverse = {false,false,false}, cubic everywhere            \
   * (spline3.inl:678-900); calc_eb: alpha 1.25 per level above unit 1, floor ebx2/2 */         \
  static void SUF##_interpolate(T* s, T* e, const tile_ctx* t, float eb_r0, float ebx20,         \
                                int radius, int compress)                                        \
  {                                                                                              \
    static const int dims[3][3][3] = {{{5, 2, 1}, {5, 1, 3}, {4, 3, 3}},                         \
                                      {{9, 3, 2}, {9, 2, 5}, {8, 5, 5}},                         \
                                      {{17, 5, 4}, {17, 4, 9}, {16, 9, 9}}};                     \
    for (int lv = 0; lv < 3; lv++) {                                                             \
      const int u = 4 >> lv;                                                                     \
      float eb_r = eb_r0, ebx2 = ebx20;                                                          \
      for (int tmp = 1; tmp < u; tmp *= 2) {                                                     \
        eb_r = (float)((double)eb_r * 1.25);                                                     \
        ebx2 = (float)((double)ebx2 / 1.25);                                                     \
      }                                                                                          \
      if ((double)ebx2 < (double)ebx20 / 2.0) {                                                  \
        ebx2 = (float)((double)ebx20 / 2.0);                                                     \
        eb_r = (float)((double)eb_r0 * 2.0);                                                     \
      }                                                                                          \
      for (int dir = 0; dir < 3; dir++)                                                          \
        SUF##_stage(s, e, t, dir, u, dims[lv][dir][0], dims[lv][dir][1], dims[lv][dir][2],       \
                    !(lv == 2 && dir == 2), eb_r, ebx2, radius, compress);                       \
    }                                                                                            \
  }                                                                                              \
                                                                                                 \
  size_t orc_spline3_c_##SUF(const T* in, size_t X, size_t Y, size_t Z, double eb, int radius,   \
                             uint16_t* codes, T* anchors, float* ol_val, uint32_t* ol_idx,       \
                             size_t ol_cap)                                                      \
  {                                                                                              \
    const float eb_r = (float)(1.0 / eb), ebx2 = (float)(eb * 2.0); /* compressor.inl:107-108 */ \
    tile_ctx t = {0, 0, 0, (unsigned)((X + 31) / 32), (unsigned)((Y + 7) / 8), (unsigned)((Z + 7) / 8), X, Y, Z}; \
    const size_t ax = (X + 7) / 8, ay = (Y + 7) / 8;                                             \
    T s[SX * SY * SZ], e[SX * SY * SZ];                                                          \
    size_t nol = 0;                                                                              \
    for (t.bz = 0; t.bz < t.gdz; t.bz++)                                                         \
      for (t.by = 0; t.by < t.gdy; t.by++)                                                       \
        for (t.bx = 0; t.bx < t.gdx; t.bx++) {                                                   \
          /* c_reset_scratch + global2shmem_33x9x9data (spline3.inl:183-203, :281-305) */       \
          for (int i = 0; i < SX * SY * SZ; i++) s[i] = 0, e[i] = 0;                             \
          for (int z = 0; z < SZ; z++)                                                           \
            for (int y = 0; y < SY; y++)                                                         \
              for (int x = 0; x < SX; x++) {                                                     \
                const size_t gx = (size_t)t.bx * 32 + x, gy = (size_t)t.by * 8 + y, gz = (size_t)t.bz * 8 + z; \
                if (x % 8 == 0 && y % 8 == 0 && z % 8 == 0) e[SIDX(x, y, z)] = (T)radius;        \
                if (gx < X && gy < Y && gz < Z) s[SIDX(x, y, z)] = in[gx + X * (gy + Y * gz)];   \
              }                                                                                  \
          /* c_gather_anchor (spline3.inl:205-220): interior points on the 8-lattice */          \
          for (int x = 0; x < 32; x += 8) {                                                      \
            const size_t gx = (size_t)t.bx * 32 + x, gy = (size_t)t.by * 8, gz = (size_t)t.bz * 8; \
            if (gx < X && gy < Y && gz < Z) anchors[gx / 8 + ax * (gy / 8 + ay * (gz / 8))] = in[gx + X * (gy + Y * gz)]; \
          }                                                                                      \
          SUF##_interpolate(s, e, &t, eb_r, ebx2, radius, 1);                                    \
          /* shmem2global_32x8x8data_with_compaction (spline3.inl:370-398) */                    \
          for (int z = 0; z < 8; z++)                                                            \
            for (int y = 0; y < 8; y++)                                                          \
              for (int x = 0; x < 32; x++) {                                                     \
                const size_t gx = (size_t)t.bx * 32 + x, gy = (size_t)t.by * 8 + y, gz = (size_t)t.bz * 8 + z; \
                if (!(gx < X && gy < Y && gz < Z)) continue;                                     \
                const size_t gid = gx + X * (gy + Y * gz);                                       \
                const T cand = e[SIDX(x, y, z)];                                                 \
                const int q = cand >= 0 && cand < 2 * radius;                                    \
                codes[gid] = q ? (uint16_t)cand : 0;                                             \
                if (!q) {                                                                        \
                  if (nol < ol_cap) ol_val[nol] = (float)cand, ol_idx[nol] = (uint32_t)gid;      \
                  nol++;                                                                         \
                }                                                                                \
              }                                                                                  \
        }                                                                                        \
    return nol;                                                                                  \
  }                                                                                              \
                                                                                                 \
  void orc_spline3_x_##SUF(const uint16_t* codes, const T* anchors, const float* ol_val,         \
                           const uint32_t* ol_idx, size_t nol, size_t X, size_t Y, size_t Z,     \
                           double eb, int radius, T* out)                                        \
  {                                                                                              \
    const float eb_r = (float)(1.0 / eb), ebx2 = (float)(eb * 2.0);                              \
    const size_t n = X * Y * Z;                                                                  \
    tile_ctx t = {0, 0, 0, (unsigned)((X + 31) / 32), (unsigned)((Y + 7) / 8), (unsigned)((Z + 7) / 8), X, Y, Z}; \
    const size_t ax = (X + 7) / 8, ay = (Y + 7) / 8, az = (Z + 7) / 8;                           \
    T s[SX * SY * SZ], e[SX * SY * SZ];                                                          \
    T* outc = out;                                                                               \
    /* outlier codes scattered onto a zero plane (GPU_scatter, spvn.cuhip.inl:66-76).  The      \
     * reference scatters into the output buffer that other tiles are writing (a race on the    \
     * +1 faces); a separate plane gives the intended semantics. */                             \
    T* ocode = (T*)calloc(n, sizeof(T));                                                         \
    for (size_t k = 0; k < nol; k++)                                                             \
      if (ol_idx[k] < n) ocode[ol_idx[k]] = (T)ol_val[k];                                        \
    for (t.bz = 0; t.bz < t.gdz; t.bz++)                                                         \
      for (t.by = 0; t.by < t.gdy; t.by++)                                                       \
        for (t.bx = 0; t.bx < t.gdx; t.bx++) {                                                   \
          /* x_reset_scratch_33x9x9data + global2shmem_fuse (spline3.inl:241-278, :309-328) */   \
          for (int z = 0; z < SZ; z++)                                                           \
            for (int y = 0; y < SY; y++)                                                         \
              for (int x = 0; x < SX; x++) {                                                     \
                const int i = SIDX(x, y, z);                                                     \
                e[i] = 0;                                                                        \
                s[i] = 0;                                                                        \
                if (x % 8 == 0 && y % 8 == 0 && z % 8 == 0) {                                    \
                  const size_t Ax = x / 8 + (size_t)t.bx * 4, Ay = y / 8 + t.by, Az = z / 8 + t.bz; \
                  if (Ax < ax && Ay < ay && Az < az) s[i] = anchors[Ax + ax * (Ay + ay * Az)];   \
                }                                                                                \
                const size_t gx = (size_t)t.bx * 32 + x, gy = (size_t)t.by * 8 + y, gz = (size_t)t.bz * 8 + z; \
                if (gx < X && gy < Y && gz < Z) {                                                \
                  const size_t gid = gx + X * (gy + Y * gz);                                     \
                  e[i] = (T)codes[gid] + ocode[gid];                                             \
                }                                                                                \
              }                                                                                  \
          SUF##_interpolate(s, e, &t, eb_r, ebx2, radius, 0);                                    \
          for (int z = 0; z < 8; z++)                                                            \
            for (int y = 0; y < 8; y++)                                                          \
              for (int x = 0; x < 32; x++) {                                                     \
                const size_t gx = (size_t)t.bx * 32 + x, gy = (size_t)t.by * 8 + y, gz = (size_t)t.bz * 8 + z; \
                if (gx < X && gy < Y && gz < Z) outc[gx + X * (gy + Y * gz)] = s[SIDX(x, y, z)]; \
              }                                                                                  \
        }                                                                                        \
    free(ocode);                                                                                 \
  }

DEFINE_SPLINE(f32, float, fabsf)
DEFINE_SPLINE(f64, double, fabs)
