/*
 * oracle.c — TEST INFRASTRUCTURE ONLY.  CPU restatement of the hot-path
 * arithmetic the reference delegates to libduckdb (duckdb_query at
 * /root/reference/src/duckdb_native.c:159, :2246), used by tests/, by
 * __graft_entry__.smoke() as the checker and by bench.py's cpu_baseline leg.
 * The product (duckdb.mbt_amd/) never links or calls this file.
 *
 * Parity anchor: libduckdb itself is not in /root/reference (it is an
 * un-vendored dependency, "latest" in .github/workflows/native-ci.yml:31-40;
 * the JS path pins @duckdb/node-api 1.4.3-r.3, package-lock.json:26-29) and is
 * not installed in this image.  The semantics restated here are DuckDB's for
 * the recognised shapes, pinned by the reference's golden fixtures
 * (src/duckdb_fixture_cases.mbt) and native tests (see tests/golden/):
 *   COUNT(*) -> BIGINT, SUM(BIGINT/INTEGER) -> HUGEINT (exact int128),
 *   MIN/MAX -> input type, '%' truncated modulo, range(N) = 0..N-1.
 *
 * Synthetic data: x_i = splitmix64(seed + start + i) mod m + add.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef __int128 i128;
#define MAXT 1024 /* threads per call: one per host CPU on the largest boxes */

uint64_t orc_splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void orc_synth_i64(int64_t *out, int64_t n, uint64_t seed, int64_t start, uint64_t m, int64_t add) {
  for (int64_t i = 0; i < n; i++) out[i] = (int64_t)(orc_splitmix64(seed + (uint64_t)(start + i)) % m) + add;
}

void orc_synth_i32(int32_t *out, int64_t n, uint64_t seed, int64_t start, uint64_t m, int64_t add) {
  for (int64_t i = 0; i < n; i++) out[i] = (int32_t)((int64_t)(orc_splitmix64(seed + (uint64_t)(start + i)) % m) + add);
}

/* ---- filter + aggregate over a materialized int64 column --------------- */
typedef struct {
  const int64_t *x;
  int64_t n;
  int64_t lo, hi;
  uint64_t count;
  i128 sum;
  int64_t mn, mx;
} fa_job;

static void *fa_run(void *p) {
  fa_job *j = (fa_job *)p;
  uint64_t c = 0;
  i128 s = 0;
  int64_t mn = INT64_MAX, mx = INT64_MIN;
  /* branch-free: the predicate becomes an all-ones/zero mask (a ~50 %
     selective branch would mispredict on every other row) */
  const int64_t lo = j->lo, hi = j->hi;
  for (int64_t i = 0; i < j->n; i++) {
    int64_t v = j->x[i];
    int64_t m = -(int64_t)((v >= lo) & (v <= hi));
    c += (uint64_t)(m & 1);
    s += (i128)(v & m);
    int64_t vmn = (v & m) | (INT64_MAX & ~m), vmx = (v & m) | (INT64_MIN & ~m);
    mn = vmn < mn ? vmn : mn;
    mx = vmx > mx ? vmx : mx;
  }
  j->count = c;
  j->sum = s;
  j->mn = mn;
  j->mx = mx;
  return NULL;
}

/* COUNT(*), SUM(x), MIN(x), MAX(x) WHERE lo <= x <= hi.  sum -> 16 bytes LE. */
void orc_filter_agg_i64(const int64_t *x, int64_t n, int64_t lo, int64_t hi, int threads, uint64_t *count,
                        void *sum16, int64_t *mn, int64_t *mx) {
  if (threads < 1) threads = 1;
  if (threads > MAXT) threads = MAXT;
  fa_job jobs[MAXT];
  pthread_t th[MAXT];
  int64_t chunk = (n + threads - 1) / threads;
  for (int t = 0; t < threads; t++) {
    int64_t b = t * chunk, e = b + chunk < n ? b + chunk : n;
    if (b > n) b = n;
    jobs[t].x = x + b;
    jobs[t].n = e - b;
    jobs[t].lo = lo;
    jobs[t].hi = hi;
    pthread_create(&th[t], NULL, fa_run, &jobs[t]);
  }
  uint64_t c = 0;
  i128 s = 0;
  int64_t a = INT64_MAX, z = INT64_MIN;
  for (int t = 0; t < threads; t++) {
    pthread_join(th[t], NULL);
    c += jobs[t].count;
    s += jobs[t].sum;
    if (jobs[t].mn < a) a = jobs[t].mn;
    if (jobs[t].mx > z) z = jobs[t].mx;
  }
  *count = c;
  memcpy(sum16, &s, 16);
  *mn = a;
  *mx = z;
}

/* ---- the same over the generator (no materialisation; full-size parity) - */
typedef struct {
  uint64_t seed, m;
  int64_t start, n, add, lo, hi;
  uint64_t count;
  i128 sum;
} sf_job;

static void *sf_run(void *p) {
  sf_job *j = (sf_job *)p;
  uint64_t c = 0;
  i128 s = 0;
  for (int64_t i = 0; i < j->n; i++) {
    int64_t v = (int64_t)(orc_splitmix64(j->seed + (uint64_t)(j->start + i)) % j->m) + j->add;
    if (v >= j->lo && v <= j->hi) {
      c++;
      s += v;
    }
  }
  j->count = c;
  j->sum = s;
  return NULL;
}

void orc_synth_filter_count(uint64_t seed, int64_t start, int64_t n, uint64_t m, int64_t add, int64_t lo, int64_t hi,
                            int threads, uint64_t *count, void *sum16) {
  if (threads < 1) threads = 1;
  if (threads > MAXT) threads = MAXT;
  sf_job jobs[MAXT];
  pthread_t th[MAXT];
  int64_t chunk = (n + threads - 1) / threads;
  for (int t = 0; t < threads; t++) {
    int64_t b = t * chunk, e = b + chunk < n ? b + chunk : n;
    if (b > n) b = n;
    jobs[t].seed = seed;
    jobs[t].m = m;
    jobs[t].start = start + b;
    jobs[t].n = e - b;
    jobs[t].add = add;
    jobs[t].lo = lo;
    jobs[t].hi = hi;
    pthread_create(&th[t], NULL, sf_run, &jobs[t]);
  }
  uint64_t c = 0;
  i128 s = 0;
  for (int t = 0; t < threads; t++) {
    pthread_join(th[t], NULL);
    c += jobs[t].count;
    s += jobs[t].sum;
  }
  *count = c;
  memcpy(sum16, &s, 16);
}

/* ---- GROUP BY small integer key, SUM(int64) as int128, COUNT(*) --------- */
typedef struct {
  const int32_t *k;
  const int64_t *v;
  int64_t n;
  int32_t kmin;
  int nk;
  uint64_t *cnt;
  i128 *sum;
} gb_job;

static void *gb_run(void *p) {
  gb_job *j = (gb_job *)p;
  if (j->nk > 64) {
    for (int64_t i = 0; i < j->n; i++) {
      int s = j->k[i] - j->kmin;
      j->cnt[s]++;
      j->sum[s] += j->v[i];
    }
    return NULL;
  }
  /* small key domain: thread-local counters in registers/stack, int64 partial
     sums flushed into the int128 totals every 2^20 rows (|v| < 2^43 cannot
     overflow an int64 partial in 2^20 additions for the C3 domain; larger
     |v| takes the exact int128 path below) */
  uint64_t cnt[64] = {0};
  int64_t part[64] = {0};
  i128 tot[64] = {0};
  int ok = 1;
  for (int64_t b = 0; b < j->n; b += 1 << 20) {
    int64_t e = b + (1 << 20) < j->n ? b + (1 << 20) : j->n;
    for (int64_t i = b; i < e && ok; i++) {
      int64_t v = j->v[i];
      if (v >= (1ll << 43) || v <= -(1ll << 43)) ok = 0;
    }
    if (!ok) break;
    for (int64_t i = b; i < e; i++) {
      int s = j->k[i] - j->kmin;
      cnt[s]++;
      part[s] += j->v[i];
    }
    for (int s = 0; s < j->nk; s++) {
      tot[s] += part[s];
      part[s] = 0;
    }
  }
  if (!ok) {
    for (int64_t i = 0; i < j->n; i++) {
      int s = j->k[i] - j->kmin;
      j->cnt[s]++;
      j->sum[s] += j->v[i];
    }
    return NULL;
  }
  for (int s = 0; s < j->nk; s++) {
    j->cnt[s] = cnt[s];
    j->sum[s] = tot[s];
  }
  return NULL;
}

/* counts[nk], sums16[nk*16] (int128 LE) */
void orc_groupby_sum_i32_i64(const int32_t *k, const int64_t *v, int64_t n, int32_t kmin, int nk, int threads,
                             uint64_t *counts, void *sums16) {
  if (threads < 1) threads = 1;
  if (threads > MAXT) threads = MAXT;
  gb_job jobs[MAXT];
  pthread_t th[MAXT];
  int64_t chunk = (n + threads - 1) / threads;
  for (int t = 0; t < threads; t++) {
    int64_t b = t * chunk, e = b + chunk < n ? b + chunk : n;
    if (b > n) b = n;
    jobs[t].k = k + b;
    jobs[t].v = v + b;
    jobs[t].n = e - b;
    jobs[t].kmin = kmin;
    jobs[t].nk = nk;
    jobs[t].cnt = (uint64_t *)calloc(nk, sizeof(uint64_t));
    jobs[t].sum = (i128 *)calloc(nk, sizeof(i128));
    pthread_create(&th[t], NULL, gb_run, &jobs[t]);
  }
  i128 *acc = (i128 *)calloc(nk, sizeof(i128));
  memset(counts, 0, nk * sizeof(uint64_t));
  for (int t = 0; t < threads; t++) {
    pthread_join(th[t], NULL);
    for (int s = 0; s < nk; s++) {
      counts[s] += jobs[t].cnt[s];
      acc[s] += jobs[t].sum[s];
    }
    free(jobs[t].cnt);
    free(jobs[t].sum);
  }
  memcpy(sums16, acc, (size_t)nk * 16);
  free(acc);
}

/* ---- the C3 GROUP BY over the generator (no materialisation) -----------
 * k_i = splitmix64(seed_k + start + i) mod nk (INT32), v_i = splitmix64(seed_v
 * + start + i) mod vm + vadd (INT64); counts[nk], sums16[nk*16] as above. */
typedef struct {
  uint64_t seed_k, seed_v, vm;
  int64_t start, n, vadd;
  int nk;
  uint64_t *cnt;
  i128 *sum;
} sg_job;

static void *sg_run(void *p) {
  sg_job *j = (sg_job *)p;
  int64_t *part = (int64_t *)calloc(j->nk, sizeof(int64_t));
  int64_t since = 0;
  for (int64_t i = 0; i < j->n; i++) {
    uint64_t r = (uint64_t)(j->start + i);
    int s = (int)(orc_splitmix64(j->seed_k + r) % (uint64_t)j->nk);
    int64_t v = (int64_t)(orc_splitmix64(j->seed_v + r) % j->vm) + j->vadd;
    j->cnt[s]++;
    part[s] += v; /* |v| < 2^62 / 2^20: flushed every 2^20 rows */
    if (++since == (1 << 20)) {
      for (int q = 0; q < j->nk; q++) j->sum[q] += part[q], part[q] = 0;
      since = 0;
    }
  }
  for (int q = 0; q < j->nk; q++) j->sum[q] += part[q];
  free(part);
  return NULL;
}

void orc_synth_groupby(uint64_t seed_k, uint64_t seed_v, int64_t start, int64_t n, int nk, uint64_t vm, int64_t vadd,
                       int threads, uint64_t *counts, void *sums16) {
  if (threads < 1) threads = 1;
  if (threads > MAXT) threads = MAXT;
  sg_job jobs[MAXT];
  pthread_t th[MAXT];
  int64_t chunk = (n + threads - 1) / threads;
  for (int t = 0; t < threads; t++) {
    int64_t b = t * chunk, e = b + chunk < n ? b + chunk : n;
    if (b > n) b = n;
    jobs[t].seed_k = seed_k;
    jobs[t].seed_v = seed_v;
    jobs[t].vm = vm;
    jobs[t].start = start + b;
    jobs[t].n = e - b;
    jobs[t].vadd = vadd;
    jobs[t].nk = nk;
    jobs[t].cnt = (uint64_t *)calloc(nk, sizeof(uint64_t));
    jobs[t].sum = (i128 *)calloc(nk, sizeof(i128));
    pthread_create(&th[t], NULL, sg_run, &jobs[t]);
  }
  i128 *acc = (i128 *)calloc(nk, sizeof(i128));
  memset(counts, 0, nk * sizeof(uint64_t));
  for (int t = 0; t < threads; t++) {
    pthread_join(th[t], NULL);
    for (int q = 0; q < nk; q++) {
      counts[q] += jobs[t].cnt[q];
      acc[q] += jobs[t].sum[q];
    }
    free(jobs[t].cnt);
    free(jobs[t].sum);
  }
  memcpy(sums16, acc, (size_t)nk * 16);
  free(acc);
}

/* ---- the C3 GROUP BY with NULL keys and two NULL-able value columns ----
 * Over the generator, row r = start + i:
 *   k = splitmix64(sd[0] + r) mod md[0] (INT32), NULL when md[1] && splitmix64(sd[1] + r) mod md[1] == 0;
 *   v = splitmix64(sd[2] + r) mod md[2] + ad[0], NULL when md[3] && splitmix64(sd[3] + r) mod md[3] == 0;
 *   w = splitmix64(sd[4] + r) mod md[4] + ad[1], NULL when md[5] && splitmix64(sd[5] + r) mod md[5] == 0.
 * DuckDB's rules (GROUP BY puts every NULL key in one group; COUNT(col), SUM,
 * MIN, MAX skip NULLs): per group g in 0..nk (g = nk: the NULL key),
 * counts[3g..] = {COUNT(*), COUNT(v), COUNT(w)}, sums16[2g..] = {SUM(v), SUM(w)}
 * as int128, mm[4g..] = {MIN(v), MAX(v), MIN(w), MAX(w)} (INT64_MAX / MIN when
 * the group has no valid value). */
typedef struct {
  const uint64_t *sd, *md;
  const int64_t *ad;
  int64_t start, n;
  int nk;
  uint64_t *cnt;
  i128 *sum;
  int64_t *mm;
} sgn_job;

static void *sgn_run(void *p) {
  sgn_job *j = (sgn_job *)p;
  const int ng = j->nk + 1;
  for (int64_t i = 0; i < j->n; i++) {
    const uint64_t r = (uint64_t)(j->start + i);
    int g = (int)(orc_splitmix64(j->sd[0] + r) % j->md[0]);
    if (j->md[1] && orc_splitmix64(j->sd[1] + r) % j->md[1] == 0) g = j->nk;
    j->cnt[3 * g]++;
    for (int c = 0; c < 2; c++) {
      const uint64_t *sd = j->sd + 2 + 2 * c, *md = j->md + 2 + 2 * c;
      if (md[1] && orc_splitmix64(sd[1] + r) % md[1] == 0) continue;
      const int64_t v = (int64_t)(orc_splitmix64(sd[0] + r) % md[0]) + j->ad[c];
      j->cnt[3 * g + 1 + c]++;
      j->sum[2 * g + c] += v;
      int64_t *m = j->mm + 4 * g + 2 * c;
      if (v < m[0]) m[0] = v;
      if (v > m[1]) m[1] = v;
    }
  }
  (void)ng;
  return NULL;
}

void orc_synth_groupby_nulls(const uint64_t *sd, const uint64_t *md, const int64_t *ad, int64_t start, int64_t n,
                             int threads, uint64_t *counts, void *sums16, int64_t *mm) {
  if (threads < 1) threads = 1;
  if (threads > MAXT) threads = MAXT;
  const int nk = (int)md[0], ng = nk + 1;
  sgn_job jobs[MAXT];
  pthread_t th[MAXT];
  int64_t chunk = (n + threads - 1) / threads;
  for (int t = 0; t < threads; t++) {
    int64_t b = t * chunk, e = b + chunk < n ? b + chunk : n;
    if (b > n) b = n;
    jobs[t].sd = sd, jobs[t].md = md, jobs[t].ad = ad;
    jobs[t].start = start + b;
    jobs[t].n = e - b;
    jobs[t].nk = nk;
    jobs[t].cnt = (uint64_t *)calloc((size_t)3 * ng, sizeof(uint64_t));
    jobs[t].sum = (i128 *)calloc((size_t)2 * ng, sizeof(i128));
    jobs[t].mm = (int64_t *)malloc((size_t)4 * ng * sizeof(int64_t));
    for (int q = 0; q < 4 * ng; q++) jobs[t].mm[q] = (q & 1) ? INT64_MIN : INT64_MAX;
    pthread_create(&th[t], NULL, sgn_run, &jobs[t]);
  }
  i128 *acc = (i128 *)calloc((size_t)2 * ng, sizeof(i128));
  memset(counts, 0, (size_t)3 * ng * sizeof(uint64_t));
  for (int q = 0; q < 4 * ng; q++) mm[q] = (q & 1) ? INT64_MIN : INT64_MAX;
  for (int t = 0; t < threads; t++) {
    pthread_join(th[t], NULL);
    for (int q = 0; q < 3 * ng; q++) counts[q] += jobs[t].cnt[q];
    for (int q = 0; q < 2 * ng; q++) acc[q] += jobs[t].sum[q];
    for (int q = 0; q < 4 * ng; q++) {
      const int64_t x = jobs[t].mm[q];
      if ((q & 1) ? x > mm[q] : x < mm[q]) mm[q] = x;
    }
    free(jobs[t].cnt);
    free(jobs[t].sum);
    free(jobs[t].mm);
  }
  memcpy(sums16, acc, (size_t)2 * ng * 16);
  free(acc);
}

/* ---- range(N) WHERE i % k = c, projected i*mul (config C1) ------------- */
int64_t orc_range_mod_select(int64_t n, int64_t k, int64_t c, int64_t mul, int64_t *out, int64_t cap) {
  int64_t w = 0;
  for (int64_t i = 0; i < n; i++)
    if (i % k == c) {
      if (w < cap) out[w] = i * mul;
      w++;
    }
  return w;
}

/* ---- SELECT x WHERE lo <= x <= hi (order-preserving compaction) --------
 * What DuckDB's filter + result materialisation produces for the selection
 * shape (SELECT x FROM t WHERE x > 24): the passing rows in row order.  Two
 * phases over contiguous per-thread chunks: count, then each thread copies its
 * passing rows to its exclusive-prefix offset (branch-free store + conditional
 * advance).  out needs room for n values; returns the count. */
typedef struct {
  const int64_t *x;
  int64_t n, lo, hi, count, off;
  int64_t *out;
} sel_job;

static void *sel_count(void *p) {
  sel_job *j = (sel_job *)p;
  int64_t c = 0;
  for (int64_t i = 0; i < j->n; i++) c += (j->x[i] >= j->lo) & (j->x[i] <= j->hi);
  j->count = c;
  return NULL;
}

static void *sel_copy(void *p) {
  sel_job *j = (sel_job *)p;
  int64_t *o = j->out + j->off;
  int64_t w = 0, junk;
  for (int64_t i = 0; i < j->n; i++) {
    const int64_t v = j->x[i];
    /* unconditional store (a cmov'd address), so the ~50 % selective
       predicate costs no mispredicted branch; past this chunk's last output
       the store goes to a scratch word, never into the next chunk */
    int64_t *d = w < j->count ? o + w : &junk;
    *d = v;
    w += (v >= j->lo) & (v <= j->hi);
  }
  (void)junk;
  return NULL;
}

int64_t orc_select_i64(const int64_t *x, int64_t n, int64_t lo, int64_t hi, int threads, int64_t *out) {
  if (threads < 1) threads = 1;
  if (threads > MAXT) threads = MAXT;
  static sel_job jobs[MAXT];
  pthread_t th[MAXT];
  int64_t chunk = (n + threads - 1) / threads;
  for (int t = 0; t < threads; t++) {
    int64_t b = t * chunk, e = b + chunk < n ? b + chunk : n;
    if (b > n) b = n;
    jobs[t].x = x + b;
    jobs[t].n = e - b;
    jobs[t].lo = lo;
    jobs[t].hi = hi;
    jobs[t].out = out;
    pthread_create(&th[t], NULL, sel_count, &jobs[t]);
  }
  int64_t off = 0;
  for (int t = 0; t < threads; t++) {
    pthread_join(th[t], NULL);
    jobs[t].off = off;
    off += jobs[t].count;
  }
  for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, sel_copy, &jobs[t]);
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  return off;
}
