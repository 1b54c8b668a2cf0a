/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C (OpenMP) restatement of the reference's APVPA PathSim semantics, the
 * same rules as pathsim_oracle.py (see its header for the reference cites):
 *   AP/PX incidences are distinct sets (DPathSim_APVPA.py:86 distinct);
 *   C[a,v] = #papers of a at v; s = colsum over ALL AP rows; g = C.s (:70-88);
 *   M[x,y] = C[x,:].C[y,:] (:90-109); score = (double)(2M)/(double)(gx+gy),
 *   one IEEE division (:51-52), 0/0 -> 0.0; targets = author rows != x in
 *   ordinal order (:18-22); top-k by (score desc, y asc).
 * Used by tests/ (medium-scale parity) and by bench.py's cpu_baseline leg
 * ("port").  Never linked into or called by the product library.
 *
 * Algorithm: row-wise Gustavson over the CSC of C with a dense per-thread
 * int64 accumulator and touched list -- the straightforward CPU port.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct {
  int64_t n_authors, n_mids;
  int64_t *c_ptr;  /* CSR of C over author rows */
  int32_t *c_col, *c_val;
  int64_t *t_ptr;  /* CSC of C (author rows only) */
  int32_t *t_row, *t_val;
  int64_t *s, *g;
  int64_t *diag;   /* M[x,x] = sum_v C[x,v]^2 (the textbook PathSim denominator term) */
} orc_state;

static int cmp_pair(const void* a, const void* b) {
  const int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
  return (x > y) - (x < y);
}

/* distinct (row, col) pairs -> sorted CSR (row_ptr n_rows+1, cols). */
static void csr_distinct(int64_t n, const int32_t* r, const int32_t* c, int64_t n_rows,
                         int64_t n_cols, int64_t** ptr_out, int32_t** col_out) {
  int64_t* key = (int64_t*)malloc(sizeof(int64_t) * (n > 0 ? n : 1));
  for (int64_t i = 0; i < n; ++i) key[i] = (int64_t)r[i] * n_cols + c[i];
  qsort(key, (size_t)n, sizeof(int64_t), cmp_pair);
  int64_t m = 0;
  for (int64_t i = 0; i < n; ++i)
    if (i == 0 || key[i] != key[i - 1]) key[m++] = key[i];
  int64_t* ptr = (int64_t*)calloc((size_t)n_rows + 1, sizeof(int64_t));
  int32_t* col = (int32_t*)malloc(sizeof(int32_t) * (m > 0 ? m : 1));
  for (int64_t i = 0; i < m; ++i) {
    ptr[key[i] / n_cols + 1]++;
    col[i] = (int32_t)(key[i] % n_cols);
  }
  for (int64_t i = 0; i < n_rows; ++i) ptr[i + 1] += ptr[i];
  free(key);
  *ptr_out = ptr;
  *col_out = col;
}

orc_state* orc_create(int64_t n_ap, const int32_t* ap_row, const int32_t* ap_col, int64_t n_px,
                      const int32_t* px_paper, const int32_t* px_mid, int64_t n_rows_all,
                      int64_t n_authors, int64_t n_papers, int64_t n_mids) {
  orc_state* st = (orc_state*)calloc(1, sizeof(orc_state));
  st->n_authors = n_authors;
  st->n_mids = n_mids;
  int64_t *ap_ptr, *px_ptr;
  int32_t *ap_c, *px_c;
  csr_distinct(n_ap, ap_row, ap_col, n_rows_all, n_papers, &ap_ptr, &ap_c);
  csr_distinct(n_px, px_paper, px_mid, n_papers, n_mids, &px_ptr, &px_c);
  /* s[v] = sum_{(p,v)} indeg(p) over ALL AP rows */
  int64_t* indeg = (int64_t*)calloc((size_t)n_papers + 1, sizeof(int64_t));
  for (int64_t j = 0; j < ap_ptr[n_rows_all]; ++j) indeg[ap_c[j]]++;
  st->s = (int64_t*)calloc((size_t)n_mids + 1, sizeof(int64_t));
  for (int64_t p = 0; p < n_papers; ++p)
    for (int64_t j = px_ptr[p]; j < px_ptr[p + 1]; ++j) st->s[px_c[j]] += indeg[p];
  free(indeg);
  /* C over author rows: dense mid accumulator per row */
  st->c_ptr = (int64_t*)calloc((size_t)n_authors + 1, sizeof(int64_t));
  int64_t* acc = (int64_t*)calloc((size_t)n_mids + 1, sizeof(int64_t));
  int32_t* touched = (int32_t*)malloc(sizeof(int32_t) * ((size_t)n_mids + 1));
  int64_t cap = 1024, nnz = 0;
  st->c_col = (int32_t*)malloc(sizeof(int32_t) * cap);
  st->c_val = (int32_t*)malloc(sizeof(int32_t) * cap);
  for (int64_t a = 0; a < n_authors; ++a) {
    int64_t nt = 0;
    for (int64_t j = ap_ptr[a]; j < ap_ptr[a + 1]; ++j) {
      const int32_t p = ap_c[j];
      for (int64_t q = px_ptr[p]; q < px_ptr[p + 1]; ++q) {
        if (acc[px_c[q]]++ == 0) touched[nt++] = px_c[q];
      }
    }
    /* ascending mid order */
    for (int64_t i = 1; i < nt; ++i) {
      int32_t v = touched[i];
      int64_t k = i - 1;
      while (k >= 0 && touched[k] > v) { touched[k + 1] = touched[k]; --k; }
      touched[k + 1] = v;
    }
    if (nnz + nt > cap) {
      while (nnz + nt > cap) cap *= 2;
      st->c_col = (int32_t*)realloc(st->c_col, sizeof(int32_t) * cap);
      st->c_val = (int32_t*)realloc(st->c_val, sizeof(int32_t) * cap);
    }
    for (int64_t i = 0; i < nt; ++i) {
      st->c_col[nnz] = touched[i];
      st->c_val[nnz] = (int32_t)acc[touched[i]];
      acc[touched[i]] = 0;
      ++nnz;
    }
    st->c_ptr[a + 1] = nnz;
  }
  free(acc);
  free(touched);
  free(ap_ptr); free(ap_c); free(px_ptr); free(px_c);
  /* g = C.s */
  st->g = (int64_t*)calloc((size_t)n_authors + 1, sizeof(int64_t));
  for (int64_t a = 0; a < n_authors; ++a) {
    int64_t gx = 0;
    for (int64_t j = st->c_ptr[a]; j < st->c_ptr[a + 1]; ++j)
      gx += (int64_t)st->c_val[j] * st->s[st->c_col[j]];
    st->g[a] = gx;
  }
  st->diag = (int64_t*)calloc((size_t)n_authors + 1, sizeof(int64_t));
  for (int64_t a = 0; a < n_authors; ++a) {
    int64_t dx = 0;
    for (int64_t j = st->c_ptr[a]; j < st->c_ptr[a + 1]; ++j)
      dx += (int64_t)st->c_val[j] * st->c_val[j];
    st->diag[a] = dx;
  }
  /* CSC of C (rows ascending within each column) */
  st->t_ptr = (int64_t*)calloc((size_t)n_mids + 1, sizeof(int64_t));
  for (int64_t j = 0; j < nnz; ++j) st->t_ptr[st->c_col[j] + 1]++;
  for (int64_t v = 0; v < n_mids; ++v) st->t_ptr[v + 1] += st->t_ptr[v];
  st->t_row = (int32_t*)malloc(sizeof(int32_t) * (nnz > 0 ? nnz : 1));
  st->t_val = (int32_t*)malloc(sizeof(int32_t) * (nnz > 0 ? nnz : 1));
  int64_t* cur = (int64_t*)malloc(sizeof(int64_t) * ((size_t)n_mids + 1));
  memcpy(cur, st->t_ptr, sizeof(int64_t) * ((size_t)n_mids + 1));
  for (int64_t a = 0; a < n_authors; ++a)
    for (int64_t j = st->c_ptr[a]; j < st->c_ptr[a + 1]; ++j) {
      const int64_t pos = cur[st->c_col[j]]++;
      st->t_row[pos] = (int32_t)a;
      st->t_val[pos] = st->c_val[j];
    }
  free(cur);
  return st;
}

int64_t orc_nnz(const orc_state* st) { return st->c_ptr[st->n_authors]; }

/* Test switches (orc_set_flags; 0 = the defaults every caller gets):
 *   ORC_FORCE_I64  int64 accumulators even when fits_i32 proves int32 suffices;
 *   ORC_NO_SKIP    no division-skip bound (every candidate is divided).
 * tests/test_oracle.py runs the oracle both ways against the numpy restatement,
 * so the shortcuts below are checked against the plain algorithm. */
#define ORC_FORCE_I64 1
#define ORC_NO_SKIP 2
static int orc_flags = 0;
void orc_set_flags(int flags) { orc_flags = flags; }
int orc_get_flags(void) { return orc_flags; }

static int fits_i32(const orc_state* st);

/* 1 when the top-k runs on int32 accumulators (fits_i32, no ORC_FORCE_I64). */
int orc_narrow(const orc_state* st) { return !(orc_flags & ORC_FORCE_I64) && fits_i32(st); }

void orc_export(const orc_state* st, int64_t* c_ptr, int32_t* c_col, int32_t* c_val, int64_t* s,
                int64_t* g) {
  const int64_t nnz = orc_nnz(st);
  if (c_ptr) memcpy(c_ptr, st->c_ptr, sizeof(int64_t) * ((size_t)st->n_authors + 1));
  if (c_col) memcpy(c_col, st->c_col, sizeof(int32_t) * (size_t)nnz);
  if (c_val) memcpy(c_val, st->c_val, sizeof(int32_t) * (size_t)nnz);
  if (s) memcpy(s, st->s, sizeof(int64_t) * (size_t)st->n_mids);
  if (g) memcpy(g, st->g, sizeof(int64_t) * (size_t)st->n_authors);
}

static int better(double s1, int32_t y1, double s2, int32_t y2) {
  return s1 > s2 || (s1 == s2 && y1 < y2);
}

/* One source row x: M[x, .] accumulated in acc (type T, all zero on entry
 * and on exit), ranked into the k slots at out_*[o ..].  A full list's k-th
 * score bounds the division from below: when 2m < kth * den * (1 - 2^-40)
 * (each side exact or within 2^-52), the rounded quotient is below kth by
 * many ulps and cannot beat it -- the division is skipped, the result is the
 * same. */
#define ORC_ROW_TOPK(NAME, T)                                                              \
  static void NAME(const orc_state* st, const int64_t* den_of, int64_t na, int64_t x,      \
                   int k, T* acc, int32_t* touched, double* ts, int32_t* ty, int64_t* tm,  \
                   int32_t* out_idx, int64_t* out_cnt, double* out_score, int64_t o) {     \
    int64_t nt = 0;                                                                         \
    for (int64_t j = st->c_ptr[x]; j < st->c_ptr[x + 1]; ++j) {                            \
      const int32_t v = st->c_col[j];                                                       \
      const T cx = (T)st->c_val[j];                                                         \
      for (int64_t q = st->t_ptr[v]; q < st->t_ptr[v + 1]; ++q) {                          \
        const int32_t y = st->t_row[q];                                                     \
        if (acc[y] == 0) touched[nt++] = y;                                                 \
        acc[y] += cx * (T)st->t_val[q];                                                     \
      }                                                                                     \
    }                                                                                       \
    int filled = 0;                                                                         \
    const int64_t dx = den_of[x];                                                           \
    const int skip_ok = !(orc_flags & ORC_NO_SKIP);                                         \
    for (int64_t t = 0; t < nt; ++t) {                                                      \
      const int32_t y = touched[t];                                                         \
      const int64_t m = (int64_t)acc[y];                                                    \
      acc[y] = 0;                                                                           \
      if (y == x) continue;                                                                 \
      const int64_t den = dx + den_of[y];                                                   \
      if (skip_ok && filled == k && den &&                                                  \
          (double)(2 * m) < ts[k - 1] * (double)den * (1.0 - 0x1p-40))                      \
        continue;                                                                           \
      const double sc = den ? (double)(2 * m) / (double)den : 0.0;                          \
      if (filled == k && !better(sc, y, ts[k - 1], ty[k - 1])) continue;                    \
      int pos = filled < k ? filled : k - 1;                                                \
      while (pos > 0 && better(sc, y, ts[pos - 1], ty[pos - 1])) {                          \
        ts[pos] = ts[pos - 1]; ty[pos] = ty[pos - 1]; tm[pos] = tm[pos - 1];                \
        --pos;                                                                              \
      }                                                                                     \
      ts[pos] = sc; ty[pos] = y; tm[pos] = m;                                               \
      if (filled < k) ++filled;                                                             \
    }                                                                                       \
    /* zero-score fill by ascending target index, self and ranked excluded */              \
    int64_t want = (na - 1) < k ? (na - 1) : k;                                             \
    for (int64_t y = 0; filled < want && y < na; ++y) {                                     \
      if (y == x) continue;                                                                 \
      int dup = 0;                                                                          \
      for (int q = 0; q < filled; ++q) if (ty[q] == y && ts[q] > 0.0) { dup = 1; break; }   \
      if (dup) continue;                                                                    \
      ts[filled] = 0.0; ty[filled] = (int32_t)y; tm[filled] = 0; ++filled;                  \
    }                                                                                       \
    for (int q = 0; q < k; ++q) {                                                           \
      if (q < filled) {                                                                     \
        out_idx[o + q] = ty[q]; out_cnt[o + q] = tm[q]; out_score[o + q] = ts[q];           \
      } else {                                                                              \
        out_idx[o + q] = -1; out_cnt[o + q] = 0; out_score[o + q] = 0.0;                    \
      }                                                                                     \
    }                                                                                       \
  }
ORC_ROW_TOPK(row_topk_i64, int64_t)
ORC_ROW_TOPK(row_topk_i32, int32_t)

/* Every M[x, y] of the author rows fits 31 bits: sum_{v in x} C[x,v] *
 * max_y C[y,v] < 2^31 for every x.  Then the accumulators are int32 (half the
 * bytes of the per-thread dense row: the scatter is a random walk over it). */
static int fits_i32(const orc_state* st) {
  const int64_t nv = st->n_mids;
  int64_t* colmax = (int64_t*)calloc((size_t)nv + 1, sizeof(int64_t));
  for (int64_t v = 0; v < nv; ++v)
    for (int64_t q = st->t_ptr[v]; q < st->t_ptr[v + 1]; ++q)
      if (st->t_val[q] > colmax[v]) colmax[v] = st->t_val[q];
  int ok = 1;
  for (int64_t x = 0; ok && x < st->n_authors; ++x) {
    int64_t b = 0;
    for (int64_t j = st->c_ptr[x]; j < st->c_ptr[x + 1]; ++j) {
      b += (int64_t)st->c_val[j] * colmax[st->c_col[j]];
      if (b >= ((int64_t)1 << 31)) { ok = 0; break; }
    }
  }
  free(colmax);
  return ok;
}

/* Top-k of source rows: rows[i] (i < n_rows) if rows != NULL, else row_begin + i.
 * use_diag != 0 replaces the reference's row-sum denominator g[x] + g[y]
 * (DPathSim_APVPA.py:51-52 with :70-88) by the textbook M[x,x] + M[y,y]. */
void orc_topk_rows(const orc_state* st, const int64_t* rows, int64_t n_rows, int64_t row_begin,
                   int k, int32_t* out_idx, int64_t* out_cnt, double* out_score, int nthreads,
                   int use_diag) {
  const int64_t na = st->n_authors;
  const int64_t* den_of = use_diag ? st->diag : st->g;
  const int narrow = !(orc_flags & ORC_FORCE_I64) && fits_i32(st);
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel
  {
    void* acc = calloc((size_t)na + 1, narrow ? sizeof(int32_t) : sizeof(int64_t));
    int32_t* touched = (int32_t*)malloc(sizeof(int32_t) * ((size_t)na + 1));
    double* ts = (double*)malloc(sizeof(double) * (size_t)k);
    int32_t* ty = (int32_t*)malloc(sizeof(int32_t) * (size_t)k);
    int64_t* tm = (int64_t*)malloc(sizeof(int64_t) * (size_t)k);
#pragma omp for schedule(dynamic, 16)
    for (int64_t i = 0; i < n_rows; ++i) {
      const int64_t x = rows ? rows[i] : row_begin + i;
      if (narrow)
        row_topk_i32(st, den_of, na, x, k, (int32_t*)acc, touched, ts, ty, tm, out_idx, out_cnt,
                     out_score, i * k);
      else
        row_topk_i64(st, den_of, na, x, k, (int64_t*)acc, touched, ts, ty, tm, out_idx, out_cnt,
                     out_score, i * k);
    }
    free(acc); free(touched); free(ts); free(ty); free(tm);
  }
}

void orc_topk(const orc_state* st, int64_t row_begin, int64_t row_end, int k, int32_t* out_idx,
              int64_t* out_cnt, double* out_score, int nthreads) {
  orc_topk_rows(st, NULL, row_end - row_begin, row_begin, k, out_idx, out_cnt, out_score,
                nthreads, 0);
}

void orc_diag(const orc_state* st, int64_t* diag) {
  memcpy(diag, st->diag, sizeof(int64_t) * (size_t)st->n_authors);
}

void orc_destroy(orc_state* st) {
  if (!st) return;
  free(st->c_ptr); free(st->c_col); free(st->c_val);
  free(st->t_ptr); free(st->t_row); free(st->t_val);
  free(st->s); free(st->g); free(st->diag);
  free(st);
}
