/* Sanitizer driver for the C oracle (oracle/pathsim_oracle.c), built by
 * `make -C oracle asan` with -fsanitize=address,undefined and run by
 * tests/test_sanitizers.py.  Random multigraph-shaped incidences (duplicates,
 * non-author AP rows, papers without venues), then create / export / top-k for
 * both denominators, k larger than the number of targets, row lists, destroy.
 * Checks g = C.s and the top-k order invariants. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef struct orc_state orc_state;
orc_state* orc_create(int64_t, const int32_t*, const int32_t*, int64_t, const int32_t*,
                      const int32_t*, int64_t, int64_t, int64_t, int64_t);
int64_t orc_nnz(const orc_state*);
void orc_export(const orc_state*, int64_t*, int32_t*, int32_t*, int64_t*, int64_t*);
void orc_topk_rows(const orc_state*, const int64_t*, int64_t, int64_t, int, int32_t*, int64_t*,
                   double*, int, int);
void orc_diag(const orc_state*, int64_t*);
void orc_destroy(orc_state*);

static uint64_t s = 88172645463325252ull;
static uint32_t rnd(uint32_t n) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (uint32_t)(s % n); }

int main(void) {
  for (int trial = 0; trial < 30; ++trial) {
    const int64_t na = 1 + rnd(300), nrows = na + rnd(20), np = 1 + rnd(500), nm = 1 + rnd(40);
    const int64_t nap = rnd(2000), npx = rnd(600);
    int32_t *ar = malloc(4 * (nap + 1)), *ac = malloc(4 * (nap + 1));
    int32_t *pp = malloc(4 * (npx + 1)), *pm = malloc(4 * (npx + 1));
    for (int64_t i = 0; i < nap; ++i) { ar[i] = rnd(nrows); ac[i] = rnd(np); }
    for (int64_t i = 0; i < npx; ++i) { pp[i] = rnd(np); pm[i] = rnd(nm); }
    orc_state* st = orc_create(nap, ar, ac, npx, pp, pm, nrows, na, np, nm);
    const int64_t nnz = orc_nnz(st);
    int64_t *cp = malloc(8 * (na + 1)), *sv = malloc(8 * nm), *g = malloc(8 * na), *dg = malloc(8 * na);
    int32_t *cc = malloc(4 * (nnz + 1)), *cv = malloc(4 * (nnz + 1));
    orc_export(st, cp, cc, cv, sv, g);
    orc_diag(st, dg);
    for (int64_t x = 0; x < na; ++x) {
      int64_t gx = 0, dx = 0;
      for (int64_t j = cp[x]; j < cp[x + 1]; ++j) { gx += (int64_t)cv[j] * sv[cc[j]]; dx += (int64_t)cv[j] * cv[j]; }
      if (gx != g[x] || dx != dg[x]) { fprintf(stderr, "FAIL g/diag\n"); return 1; }
    }
    const int k = 1 + rnd(2 * (int)na + 3);
    const int64_t nr = 1 + rnd(na);
    int64_t* rows = malloc(8 * nr);
    for (int64_t i = 0; i < nr; ++i) rows[i] = rnd(na);
    int32_t* idx = malloc(4 * nr * k);
    int64_t* cnt = malloc(8 * nr * k);
    double* sc = malloc(8 * nr * k);
    for (int den = 0; den < 2; ++den) {
      orc_topk_rows(st, rows, nr, 0, k, idx, cnt, sc, 2, den);
      for (int64_t i = 0; i < nr; ++i)
        for (int q = 1; q < k; ++q) {
          const int64_t e = i * k + q;
          if (idx[e] < 0) continue;
          if (idx[e - 1] < 0 || sc[e] > sc[e - 1] || (sc[e] == sc[e - 1] && idx[e] <= idx[e - 1]) ||
              idx[e] == rows[i]) { fprintf(stderr, "FAIL order\n"); return 1; }
        }
    }
    orc_destroy(st);
    free(ar); free(ac); free(pp); free(pm); free(cp); free(sv); free(g); free(dg); free(cc);
    free(cv); free(rows); free(idx); free(cnt); free(sc);
  }
  printf("oracle asan ok\n");
  return 0;
}
