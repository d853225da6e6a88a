/*
 * dgs_oracle.c -- CPU restatement of the DGS sampling / relabel / gather path.
 * TEST INFRASTRUCTURE ONLY (see dgs_oracle.h).  Compile with -ffp-contract=off and without
 * -ffast-math: every float operation below must round exactly once, as written.
 */
#include "dgs_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ======================================================================================
 * Philox4x32-10 with curand's state machine.
 * curand_kernel.h: curand_init(seed, subsequence, offset) sets key = seed, ctr = 0, then
 * skipahead_sequence(subsequence) adds it to ctr.{z,w} and skipahead(offset) advances
 * ctr.{x..w}; curand() returns output[STATE++] and regenerates after 4 words.
 * Used by the reference at rowwise_sampling.cu:62-63,86,122,133 and
 * rowwise_sampling_bias.cu:90-92,113,119,167-169,208.
 * ==================================================================================== */
#define PHILOX_W32_0 0x9E3779B9u
#define PHILOX_W32_1 0xBB67AE85u
#define PHILOX_M4x32_0 0xD2511F53u
#define PHILOX_M4x32_1 0xCD9E8D57u

void oracle_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
  uint32_t k0 = key_in[0], k1 = key_in[1];
  for (int r = 0; r < 10; ++r) {
    if (r > 0) {
      k0 += PHILOX_W32_0;
      k1 += PHILOX_W32_1;
    }
    uint64_t p0 = (uint64_t)PHILOX_M4x32_0 * c0;
    uint64_t p1 = (uint64_t)PHILOX_M4x32_1 * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0;
    uint32_t n1 = lo1;
    uint32_t n2 = hi0 ^ c3 ^ k1;
    uint32_t n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

static void philox_incr(oracle_philox_t *st, uint64_t n) {
  /* Philox_State_Incr(state, n): 128-bit counter += n */
  uint32_t nlo = (uint32_t)n, nhi = (uint32_t)(n >> 32);
  st->ctr[0] += nlo;
  if (st->ctr[0] < nlo) nhi++;
  st->ctr[1] += nhi;
  if (nhi <= st->ctr[1]) return;
  if (++st->ctr[2]) return;
  ++st->ctr[3];
}

static void philox_incr_hi(oracle_philox_t *st, uint64_t n) {
  /* Philox_State_Incr_hi(state, n): counter.{z,w} += n */
  uint32_t nlo = (uint32_t)n, nhi = (uint32_t)(n >> 32);
  st->ctr[2] += nlo;
  if (st->ctr[2] < nlo) nhi++;
  st->ctr[3] += nhi;
}

static void philox_incr1(oracle_philox_t *st) {
  if (++st->ctr[0]) return;
  if (++st->ctr[1]) return;
  if (++st->ctr[2]) return;
  ++st->ctr[3];
}

void oracle_curand_init(uint64_t seed, uint64_t subsequence, uint64_t offset,
                        oracle_philox_t *st) {
  memset(st, 0, sizeof(*st));
  st->key[0] = (uint32_t)seed;
  st->key[1] = (uint32_t)(seed >> 32);
  st->state = 0;
  philox_incr_hi(st, subsequence);
  oracle_philox4x32_10(st->ctr, st->key, st->output);
  /* skipahead(offset) */
  st->state += (uint32_t)(offset & 3);
  uint64_t n = offset / 4;
  if (st->state > 3) {
    n += 1;
    st->state -= 4;
  }
  philox_incr(st, n);
  oracle_philox4x32_10(st->ctr, st->key, st->output);
}

uint32_t oracle_curand(oracle_philox_t *st) {
  uint32_t ret = st->output[st->state & 3];
  st->state++;
  if (st->state == 4) {
    philox_incr1(st);
    oracle_philox4x32_10(st->ctr, st->key, st->output);
    st->state = 0;
  }
  return ret;
}

/* curand_uniform: x * CURAND_2POW32_INV + CURAND_2POW32_INV/2 with CURAND_2POW32_INV = 2^-32
 * (the product is exact, so FMA contraction cannot change the result). */
static inline float curand_uniform_from(uint32_t x) {
  return (float)x * 2.3283064365386963e-10f + 1.1641532182693481e-10f;
}

float oracle_curand_uniform(oracle_philox_t *st) { return curand_uniform_from(oracle_curand(st)); }

uint32_t oracle_philox_draw(uint64_t seed, uint64_t subsequence, uint64_t j) {
  uint32_t ctr[4] = {(uint32_t)(j >> 2), (uint32_t)(j >> 34), (uint32_t)subsequence,
                     (uint32_t)(subsequence >> 32)};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t out[4];
  oracle_philox4x32_10(ctr, key, out);
  return out[j & 3];
}

/* ======================================================================================
 * std::mt19937_64 (context/context.h:9-10,17; libstdc++'s full-range
 * uniform_int_distribution<uint64_t> returns the raw engine output).
 * ==================================================================================== */
#define MT_NN 312
#define MT_MM 156
#define MT_MATRIX_A 0xB5026F5AA96619E9ULL
#define MT_UM 0xFFFFFFFF80000000ULL
#define MT_LM 0x7FFFFFFFULL

void oracle_mt64_seed(oracle_mt64_t *g, uint64_t seed) {
  g->mt[0] = seed;
  for (int i = 1; i < MT_NN; i++)
    g->mt[i] = 6364136223846793005ULL * (g->mt[i - 1] ^ (g->mt[i - 1] >> 62)) + (uint64_t)i;
  g->idx = MT_NN;
}

uint64_t oracle_mt64_next(oracle_mt64_t *g) {
  if (g->idx >= MT_NN) {
    for (int i = 0; i < MT_NN; i++) {
      uint64_t x = (g->mt[i] & MT_UM) | (g->mt[(i + 1) % MT_NN] & MT_LM);
      uint64_t xa = x >> 1;
      if (x & 1ULL) xa ^= MT_MATRIX_A;
      g->mt[i] = g->mt[(i + MT_MM) % MT_NN] ^ xa;
    }
    g->idx = 0;
  }
  uint64_t x = g->mt[g->idx++];
  x ^= (x >> 29) & 0x5555555555555555ULL;
  x ^= (x << 17) & 0x71D67FFFEDA60000ULL;
  x ^= (x << 37) & 0xFFF7EEE000000000ULL;
  x ^= (x >> 43);
  return x;
}

/* ======================================================================================
 * A-Res key.  The reference uses key = __powf(curand_uniform(), 1/p)
 * (rowwise_sampling_bias.cu:113,119); __powf is a fast-math approximation whose bits are not
 * reproducible off NVIDIA hardware.  DGS-AMD defines key = log2(u) / p (a monotone transform
 * of u^(1/p), so the same A-Res selection distribution) with the fixed-operation log2
 * below; p <= 0 (or NaN) gives -inf.  The HIP kernels evaluate the same operation sequence.
 * ==================================================================================== */
float oracle_log2f(float u) {
  uint32_t b;
  memcpy(&b, &u, 4);
  int32_t e = (int32_t)((b >> 23) & 0xFFu) - 127;
  uint32_t mb = (b & 0x007FFFFFu) | 0x3F800000u;
  float m;
  memcpy(&m, &mb, 4);
  if (m > 1.41421356f) {
    m = m * 0.5f;
    e += 1;
  }
  float f = m - 1.0f;
  float s = f / (2.0f + f);
  float s2 = s * s;
  float q = fmaf(s2, 0.11111111f, 0.14285715f);
  q = fmaf(s2, q, 0.2f);
  q = fmaf(s2, q, 0.33333334f);
  q = fmaf(s2, q, 1.0f);
  float t = 2.0f * s;
  float ln = t * q;
  return fmaf(ln, 1.44269504f, (float)e);
}

float oracle_ares_key(float u, float p) {
  if (!(p > 0.0f)) return -INFINITY;
  return oracle_log2f(u) / p;
}

/* vectorised oracle_ares_key (test helper) */
void oracle_ares_keys(const float *u, const float *p, float *out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) out[i] = oracle_ares_key(u[i], p[i]);
}

static inline int ares_better(float ka, int64_t ia, float kb, int64_t ib) {
  return ka > kb || (ka == kb && ia < ib);
}

/* ======================================================================================
 * Uniform row-wise sampling: rowwise_sampling.cu:16-45 (sub-indptr), :47-104 (K2, without
 * replacement, reservoir with atomicMax slots), :106-141 (K3, with replacement).
 * One block of 128 threads per row, grid = S: the RNG stream of thread t for row r is
 * (key = launch_seed*S + r, subsequence t, offset 0); thread t makes its j-th draw for
 * idx = k + t + 128j (K2) or idx = t + 128j (K3).  The P2P variants
 * (rowwise_sampling_p2p.cu:19-140,239-263) use the same grid and RNG coordinates, so the
 * cached and uncached samplers produce identical output.
 * ==================================================================================== */
static int64_t sample_uniform_row(int64_t r, int64_t S, int64_t row, const int64_t *indptr,
                                  const int64_t *indices, int64_t k, int replace,
                                  uint64_t launch_seed, int64_t out_off, int64_t *out_row,
                                  int64_t *out_col, int64_t *slot_scratch) {
  const int64_t begin = indptr[row];
  const int64_t deg = indptr[row + 1] - begin;
  const uint64_t key = launch_seed * (uint64_t)S + (uint64_t)r;
  if (replace) {
    if (deg == 0) return 0;
    for (int64_t idx = 0; idx < k; idx++) {
      uint32_t x = oracle_philox_draw(key, (uint64_t)(idx % 128), (uint64_t)(idx / 128));
      int64_t edge = (int64_t)x % deg;
      out_row[out_off + idx] = row;
      out_col[out_off + idx] = indices[begin + edge];
    }
    return k;
  }
  if (deg <= k) {
    for (int64_t idx = 0; idx < deg; idx++) {
      out_row[out_off + idx] = row;
      out_col[out_off + idx] = indices[begin + idx];
    }
    return deg;
  }
  int64_t *slot = slot_scratch;
  for (int64_t s = 0; s < k; s++) slot[s] = s;
  uint32_t kk[2] = {(uint32_t)key, (uint32_t)(key >> 32)};
  /* draw j of thread t serves idx = k + t + 128 j; one Philox call covers j = 4q..4q+3 */
  for (int64_t q = 0; k + 512 * q < deg; q++) {
    for (int64_t t = 0; t < 128; t++) {
      int64_t base = k + t + 512 * q;
      if (base >= deg) break;
      uint32_t ctr[4] = {(uint32_t)q, (uint32_t)((uint64_t)q >> 32), (uint32_t)t, 0u};
      uint32_t o4[4];
      oracle_philox4x32_10(ctr, kk, o4);
      for (int w = 0; w < 4; w++) {
        int64_t idx = base + 128 * w;
        if (idx >= deg) break;
        uint32_t num = o4[w] % (uint32_t)(idx + 1);
        if ((int64_t)num < k && slot[num] < idx) slot[num] = idx;
      }
    }
  }
  for (int64_t s = 0; s < k; s++) {
    out_row[out_off + s] = row;
    out_col[out_off + s] = indices[begin + slot[s]];
  }
  return k;
}

static int64_t row_count(int64_t deg, int64_t k, int replace) {
  if (replace) return deg == 0 ? 0 : k;
  return deg < k ? deg : k;
}

int64_t oracle_sample_uniform(const int64_t *seeds, int64_t S, const int64_t *indptr,
                              const int64_t *indices, int64_t k, int replace,
                              uint64_t launch_seed, int64_t *out_row, int64_t *out_col) {
  int64_t *slot = (int64_t *)malloc(sizeof(int64_t) * (size_t)(k > 0 ? k : 1));
  int64_t off = 0;
  for (int64_t r = 0; r < S; r++) {
    off += sample_uniform_row(r, S, seeds[r], indptr, indices, k, replace, launch_seed, off,
                              out_row, out_col, slot);
  }
  free(slot);
  return off;
}

int oracle_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

int64_t oracle_sample_uniform_omp(const int64_t *seeds, int64_t S, const int64_t *indptr,
                                  const int64_t *indices, int64_t k, int replace,
                                  uint64_t launch_seed, int64_t *out_row, int64_t *out_col,
                                  int nthreads) {
  int64_t *offs = (int64_t *)malloc(sizeof(int64_t) * (size_t)(S + 1));
  offs[0] = 0;
  for (int64_t r = 0; r < S; r++) {
    int64_t row = seeds[r];
    offs[r + 1] = offs[r] + row_count(indptr[row + 1] - indptr[row], k, replace);
  }
#ifdef _OPENMP
#pragma omp parallel num_threads(nthreads > 0 ? nthreads : omp_get_max_threads())
#endif
  {
    int64_t *slot = (int64_t *)malloc(sizeof(int64_t) * (size_t)(k > 0 ? k : 1));
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 256)
#endif
    for (int64_t r = 0; r < S; r++)
      sample_uniform_row(r, S, seeds[r], indptr, indices, k, replace, launch_seed, offs[r],
                         out_row, out_col, slot);
    free(slot);
  }
  int64_t nnz = offs[S];
  free(offs);
  (void)nthreads;
  return nnz;
}

/* ======================================================================================
 * Biased row-wise sampling: rowwise_sampling_bias.cu:16-60 (sub/temp indptr), :62-146 (K5,
 * A-Res without replacement), :148-224 (K6, CDF with replacement), launch :250-280.
 * Grid = ceil(S/16) blocks of (32 x 4) threads; warp w of block b handles rows
 * 16b + w + 4m (m = 0..3) and its 32 RNG states persist across those rows.
 * K5: thread (w,l) stream (key = launch_seed*G + b, subsequence 32w + l); lane l draws once
 *     per edge i = l (mod 32), i < deg, but only for rows with deg > k; the k best edges by
 *     (key desc, index asc) are written in that order (WarpSelect writeOutV order).
 * K6: subsequence 4w + l (the reference computes threadIdx.y*BLOCK_WARPS + threadIdx.x,
 *     :168-169; reproduced as is); per row with deg > 0 the CDF is built 32 edges at a time
 *     with a Kogge-Stone inclusive scan whose lane 0 first adds the previous chunk's
 *     aggregate and clamps at 0 (:185-202); pick idx = l (mod 32) draws u, r = u * cdf[deg-1],
 *     item = min(cub::UpperBound(cdf, deg, r), deg - 1) (:205-213).
 * ==================================================================================== */
typedef struct {
  float key;
  int64_t idx;
} ares_entry;

static void topk_insert(ares_entry *buf, int64_t *cnt, int64_t k, float key, int64_t idx) {
  int64_t c = *cnt;
  if (c == k && !ares_better(key, idx, buf[k - 1].key, buf[k - 1].idx)) return;
  int64_t pos = c == k ? k - 1 : c;
  while (pos > 0 && ares_better(key, idx, buf[pos - 1].key, buf[pos - 1].idx)) {
    buf[pos] = buf[pos - 1];
    pos--;
  }
  buf[pos].key = key;
  buf[pos].idx = idx;
  if (c < k) *cnt = c + 1;
}

static int64_t cub_upper_bound(const float *a, int64_t n, float val) {
  /* cub::UpperBound (cub/util_device.cuh / thread_search.cuh) */
  int64_t retval = 0;
  while (n > 0) {
    int64_t half = n >> 1;
    if (val < a[retval + half]) {
      n = half;
    } else {
      retval = retval + (half + 1);
      n = n - (half + 1);
    }
  }
  return retval;
}

static float fmax_cuda(float a, float b) { return fmaxf(a, b); }

static void build_cdf(const float *p, int64_t deg, float *cdf) {
  float agg = 0.0f;
  int64_t max_iter = (1 + (deg - 1) / 32) * 32;
  for (int64_t base = 0; base < max_iter; base += 32) {
    float v[32], nv[32];
    for (int l = 0; l < 32; l++) {
      int64_t idx = base + l;
      float td = idx < deg ? p[idx] : 0.0f;
      if (l == 0) td = td + agg;
      v[l] = fmax_cuda(td, 0.0f);
    }
    for (int s = 0; s < 5; s++) {
      int off = 1 << s;
      for (int l = 0; l < 32; l++) nv[l] = l >= off ? v[l - off] + v[l] : v[l];
      memcpy(v, nv, sizeof(v));
    }
    agg = v[31];
    for (int l = 0; l < 32; l++)
      if (base + l < deg) cdf[base + l] = v[l];
  }
}

/* One 16-row block b of K5 / K6 (4 warp chains of rows b*16 + w + 4m).  buf: k entries,
 * cdf: max_deg floats (scratch of the calling thread). */
static void sample_bias_block(int64_t b, const int64_t *seeds, int64_t S, int64_t G,
                              const int64_t *indptr, const int64_t *indices, const float *probs,
                              int64_t k, int replace, uint64_t launch_seed, const int64_t *offs,
                              int64_t *out_row, int64_t *out_col, ares_entry *buf, float *cdf) {
  oracle_philox_t st[32];
  const uint64_t key = launch_seed * (uint64_t)G + (uint64_t)b;
  const int64_t last_row = (b + 1) * 16 < S ? (b + 1) * 16 : S;
  for (int w = 0; w < 4; w++) {
    for (int l = 0; l < 32; l++)
      oracle_curand_init(key, replace ? (uint64_t)(4 * w + l) : (uint64_t)(32 * w + l), 0,
                         &st[l]);
    for (int64_t r = b * 16 + w; r < last_row; r += 4) {
      const int64_t row = seeds[r];
      const int64_t begin = indptr[row];
      const int64_t deg = indptr[row + 1] - begin;
      const int64_t o = offs[r];
      if (!replace) {
        if (deg > k) {
          int64_t cnt = 0;
          for (int64_t i = 0; i < deg; i++) {
            float u = oracle_curand_uniform(&st[i % 32]);
            float key_i = oracle_ares_key(u, probs[begin + i]);
            topk_insert(buf, &cnt, k, key_i, i);
          }
          for (int64_t j = 0; j < k; j++) {
            out_row[o + j] = row;
            out_col[o + j] = indices[begin + buf[j].idx];
          }
        } else {
          for (int64_t i = 0; i < deg; i++) {
            out_row[o + i] = row;
            out_col[o + i] = indices[begin + i];
          }
        }
      } else if (deg > 0) {
        build_cdf(probs + begin, deg, cdf);
        const float sum = cdf[deg - 1];
        for (int64_t idx = 0; idx < k; idx++) {
          float u = oracle_curand_uniform(&st[idx % 32]);
          float rnd = u * sum;
          int64_t item = cub_upper_bound(cdf, deg, rnd);
          if (item > deg - 1) item = deg - 1;
          out_row[o + idx] = row;
          out_col[o + idx] = indices[begin + item];
        }
      }
    }
  }
}

/* offs[0..S] (output offsets) and the largest degree among the seeds */
static int64_t *bias_offsets(const int64_t *seeds, int64_t S, const int64_t *indptr, int64_t k,
                             int replace, int64_t *max_deg) {
  int64_t *offs = (int64_t *)malloc(sizeof(int64_t) * (size_t)(S + 1));
  offs[0] = 0;
  *max_deg = 0;
  for (int64_t r = 0; r < S; r++) {
    int64_t row = seeds[r];
    int64_t deg = indptr[row + 1] - indptr[row];
    if (deg > *max_deg) *max_deg = deg;
    offs[r + 1] = offs[r] + row_count(deg, k, replace);
  }
  return offs;
}

int64_t oracle_sample_bias(const int64_t *seeds, int64_t S, const int64_t *indptr,
                           const int64_t *indices, const float *probs, int64_t k, int replace,
                           uint64_t launch_seed, int64_t *out_row, int64_t *out_col) {
  return oracle_sample_bias_omp(seeds, S, indptr, indices, probs, k, replace, launch_seed,
                                out_row, out_col, 1);
}

/* Blocks are independent RNG streams (key = seed * G + b), so they run in parallel. */
int64_t oracle_sample_bias_omp(const int64_t *seeds, int64_t S, const int64_t *indptr,
                               const int64_t *indices, const float *probs, int64_t k,
                               int replace, uint64_t launch_seed, int64_t *out_row,
                               int64_t *out_col, int nthreads) {
  int64_t max_deg = 0;
  int64_t *offs = bias_offsets(seeds, S, indptr, k, replace, &max_deg);
  const int64_t G = (S + 15) / 16;
#ifdef _OPENMP
#pragma omp parallel num_threads(nthreads > 0 ? nthreads : omp_get_max_threads())
#endif
  {
    ares_entry *buf = (ares_entry *)malloc(sizeof(ares_entry) * (size_t)(k > 0 ? k : 1));
    float *cdf = (float *)malloc(sizeof(float) * (size_t)(max_deg > 0 ? max_deg : 1));
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 4)
#endif
    for (int64_t b = 0; b < G; b++)
      sample_bias_block(b, seeds, S, G, indptr, indices, probs, k, replace, launch_seed, offs,
                        out_row, out_col, buf, cdf);
    free(buf);
    free(cdf);
  }
  int64_t nnz = offs[S];
  free(offs);
  (void)nthreads;
  return nnz;
}

/* ======================================================================================
 * Unique + relabel: tensor_relabel.cu:82-159 (Unique), :161-180 (Relabel), :182-205 driver.
 * unique = ids of cat(mapping) in first-occurrence order (the table keeps the minimum
 * position per key via atomicMin, :28, and flags SearchForValue(in[i]) == i, :123);
 * relabeled[i] = position of req[i] in unique, or -1 when absent (:47-61).
 * ==================================================================================== */
typedef struct {
  int64_t *keys;
  int64_t *vals;
  uint64_t mask;
} i64map;

static uint64_t mix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}

static void i64map_init(i64map *m, int64_t n) {
  uint64_t cap = 16;
  while (cap < (uint64_t)(2 * n + 1)) cap <<= 1;
  m->keys = (int64_t *)malloc(sizeof(int64_t) * cap);
  m->vals = (int64_t *)malloc(sizeof(int64_t) * cap);
  for (uint64_t i = 0; i < cap; i++) m->keys[i] = INT64_MIN;
  m->mask = cap - 1;
}

static void i64map_free(i64map *m) {
  free(m->keys);
  free(m->vals);
}

/* returns pointer to value slot; *inserted set if key was new */
static int64_t *i64map_get(i64map *m, int64_t key, int *inserted) {
  uint64_t pos = mix64((uint64_t)key) & m->mask;
  while (1) {
    if (m->keys[pos] == key) {
      *inserted = 0;
      return &m->vals[pos];
    }
    if (m->keys[pos] == INT64_MIN) {
      m->keys[pos] = key;
      *inserted = 1;
      return &m->vals[pos];
    }
    pos = (pos + 1) & m->mask;
  }
}

static const int64_t *i64map_find(const i64map *m, int64_t key) {
  uint64_t pos = mix64((uint64_t)key) & m->mask;
  while (1) {
    if (m->keys[pos] == key) return &m->vals[pos];
    if (m->keys[pos] == INT64_MIN) return NULL;
    pos = (pos + 1) & m->mask;
  }
}

int64_t oracle_relabel(const int64_t *mapping, int64_t n_map, const int64_t *req, int64_t n_req,
                       int64_t *unique_out, int64_t *relabeled_out) {
  i64map m;
  i64map_init(&m, n_map);
  int64_t u = 0;
  for (int64_t i = 0; i < n_map; i++) {
    int ins;
    int64_t *v = i64map_get(&m, mapping[i], &ins);
    if (ins) {
      *v = u;
      unique_out[u++] = mapping[i];
    }
  }
  for (int64_t i = 0; i < n_req; i++) {
    const int64_t *v = i64map_find(&m, req[i]);
    relabeled_out[i] = v ? *v : -1;
  }
  i64map_free(&m);
  return u;
}

/* ======================================================================================
 * Multi-hop node-classification sample: sampler.cc:14-36 (uniform), :38-62 (bias),
 * :146-166.  Hop loop runs i = L-1 .. 0 with fan_out[i]; one launch seed per hop.
 * ==================================================================================== */
void oracle_nc_bounds(int64_t B, const int64_t *fan_out, int L, int64_t *frontier_cap,
                      int64_t *edge_cap) {
  int64_t s = B;
  for (int i = L - 1; i >= 0; i--) {
    int64_t e = s * fan_out[i];
    edge_cap[L - 1 - i] = e;
    s = s + e;
    frontier_cap[L - 1 - i] = s;
  }
}

void oracle_node_classification_sample(const int64_t *seeds, int64_t B, const int64_t *indptr,
                                       const int64_t *indices, const float *probs,
                                       const int64_t *fan_out, int L, int replace,
                                       const uint64_t *launch_seeds, int64_t **frontiers,
                                       int64_t **rows, int64_t **cols, int64_t *sizes_out) {
  const int64_t *cur = seeds;
  int64_t S = B;
  for (int h = 0; h < L; h++) {
    int64_t k = fan_out[L - 1 - h];
    int64_t cap = S * k;
    int64_t *coo_row = (int64_t *)malloc(sizeof(int64_t) * (size_t)(cap > 0 ? cap : 1));
    int64_t nnz;
    if (probs)
      nnz = oracle_sample_bias(cur, S, indptr, indices, probs, k, replace, launch_seeds[h],
                               coo_row, cols[h]);
    else
      nnz = oracle_sample_uniform(cur, S, indptr, indices, k, replace, launch_seeds[h],
                                  coo_row, cols[h]);
    /* relabel({seeds, coo_col}, {coo_row, coo_col}) */
    int64_t nm = S + nnz;
    int64_t *mapping = (int64_t *)malloc(sizeof(int64_t) * (size_t)(nm > 0 ? nm : 1));
    memcpy(mapping, cur, sizeof(int64_t) * (size_t)S);
    memcpy(mapping + S, cols[h], sizeof(int64_t) * (size_t)nnz);
    int64_t *req = (int64_t *)malloc(sizeof(int64_t) * (size_t)(2 * nnz > 0 ? 2 * nnz : 1));
    memcpy(req, coo_row, sizeof(int64_t) * (size_t)nnz);
    memcpy(req + nnz, cols[h], sizeof(int64_t) * (size_t)nnz);
    int64_t *rel = (int64_t *)malloc(sizeof(int64_t) * (size_t)(2 * nnz > 0 ? 2 * nnz : 1));
    int64_t U = oracle_relabel(mapping, nm, req, 2 * nnz, frontiers[h], rel);
    memcpy(rows[h], rel, sizeof(int64_t) * (size_t)nnz);
    memcpy(cols[h], rel + nnz, sizeof(int64_t) * (size_t)nnz);
    sizes_out[3 * h + 0] = S;
    sizes_out[3 * h + 1] = U;
    sizes_out[3 * h + 2] = nnz;
    free(coo_row);
    free(mapping);
    free(req);
    free(rel);
    cur = frontiers[h];
    S = U;
  }
}

/* ======================================================================================
 * Cache extraction: utils.cu:12-42 (ExtractIndptr: degrees -> exclusive scan) and
 * :44-101 (ExtractEdgeData: row-wise copy of edge data into the sub-CSR).
 * ==================================================================================== */
void oracle_extract_indptr(const int64_t *nids, int64_t n, const int64_t *indptr,
                           int64_t *sub_indptr) {
  int64_t acc = 0;
  for (int64_t i = 0; i < n; i++) {
    sub_indptr[i] = acc;
    acc += indptr[nids[i] + 1] - indptr[nids[i]];
  }
  sub_indptr[n] = acc;
}

void oracle_extract_edge_data(const int64_t *nids, int64_t n, const int64_t *indptr,
                              const int64_t *sub_indptr, const void *edge_data, int64_t elsize,
                              void *sub_edge_data) {
  const char *src = (const char *)edge_data;
  char *dst = (char *)sub_edge_data;
  for (int64_t i = 0; i < n; i++) {
    int64_t b = indptr[nids[i]], d = indptr[nids[i] + 1] - b;
    memcpy(dst + sub_indptr[i] * elsize, src + b * elsize, (size_t)(d * elsize));
  }
}

/* ======================================================================================
 * Gather: feature_ops.cu:140-210 (GetFeaturesCUDA / _IndexKernel) and the P2P gather
 * :12-138 -- both are out[i, :] = data[nids[i], :], a byte copy.
 * ==================================================================================== */
void oracle_index_select(const void *data, int64_t row_bytes, const int64_t *nids, int64_t n,
                         void *out, int nthreads) {
  const char *src = (const char *)data;
  char *dst = (char *)out;
#ifdef _OPENMP
#pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : omp_get_max_threads())
#endif
  for (int64_t i = 0; i < n; i++)
    memcpy(dst + i * row_bytes, src + nids[i] * row_bytes, (size_t)row_bytes);
  (void)nthreads;
}

/* ======================================================================================
 * Heat propagation: preprocess_heat.cu:14-33 (uniform), :58-98 (bias), drivers :35-56 and
 * :100-121.  The reference accumulates with float atomics (order-nondeterministic); the
 * oracle accumulates in seed/edge order, so comparisons use a tolerance.  The biased
 * driver processes seeds.numel() - 1 seeds (:107); reproduced as is.
 * ==================================================================================== */
void oracle_frontier_heat(const int64_t *seeds, int64_t n, const int64_t *indptr,
                          const int64_t *indices, const float *seeds_heat, int64_t num_picks,
                          int64_t indptr_diff, int64_t num_nodes, float *frontier_heat) {
  for (int64_t i = 0; i < num_nodes; i++) frontier_heat[i] = 0.0f;
  for (int64_t s = 0; s < n; s++) {
    int64_t row = seeds[s];
    int64_t b = indptr[row] - indptr_diff, e = indptr[row + 1] - indptr_diff, deg = e - b;
    for (int64_t i = 0; i < deg; i++) {
      float m = seeds_heat[row] * (float)num_picks / (float)deg;
      float msg = (1.0f < m) ? 1.0f : m;
      frontier_heat[indices[b + i]] += msg;
    }
  }
}

void oracle_frontier_heat_with_bias(const int64_t *seeds, int64_t n, const int64_t *indptr,
                                    const int64_t *indices, const float *probs,
                                    const float *seeds_heat, int64_t num_picks,
                                    int64_t indptr_diff, int64_t num_nodes,
                                    float *frontier_heat) {
  for (int64_t i = 0; i < num_nodes; i++) frontier_heat[i] = 0.0f;
  for (int64_t s = 0; s < n - 1; s++) {
    int64_t row = seeds[s];
    int64_t b = indptr[row] - indptr_diff, e = indptr[row + 1] - indptr_diff, deg = e - b;
    float psum = 0.0f;
    for (int64_t i = 0; i < deg; i++) psum += probs[b + i];
    for (int64_t i = 0; i < deg; i++) {
      float m = seeds_heat[row] * (float)num_picks * (probs[b + i] / psum);
      float msg = (1.0f < m) ? 1.0f : m;
      frontier_heat[indices[b + i]] += msg;
    }
  }
}
