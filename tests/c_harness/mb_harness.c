/*
 * mb_harness.c — drives libduckdb_mb_amd.so through include/duckdb_mb.h the
 * way MoonBit's native backend does (src/moon.pkg links the stub library;
 * src/duckdb_native.mbt calls the symbols), with a stand-in for the MoonBit
 * runtime: a STRONG moonbit_make_bytes_raw that tags every object it makes.
 * The library's own allocator is weak, so every Bytes it returns must carry
 * this runtime's tag — the property INTEGRATION.md relies on.
 *
 *   mb_harness cpu          host-constant queries only (mbx_allow_no_gpu)
 *   mb_harness gpu <rows>   C2 on the device: COUNT(*) WHERE x > 24, appender,
 *                           Arrow int64 getter; prints "count=<n>"
 *   mb_harness c1 [reps]    C1 through the per-cell query loop and the stream
 *                           chunk loop: one JSON line
 *   mb_harness c4 <rows>    C4 through the row-wise Appender + Arrow getter:
 *                           one JSON line (ingest rows/s, read-back GB/s)
 *   mb_harness c4chunk <rows>  the same with the ingest through 2048-row data
 *                           chunks (duckdb_mb_append_data_chunk)
 *   mb_harness sqlfile <f>  every line of f as a query, a prepared statement
 *                           and every result cell (sanitizer runs, no GPU)
 * Exit status 0 = every check passed.
 */
#define _POSIX_C_SOURCE 199309L
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "duckdb_mb.h"

/* ---- fake MoonBit runtime: {int32 rc; uint32 meta} header + payload ---- */
#define FAKE_RC 0x4D42 /* "MB" */
static long g_made = 0;
/* Like the runtime's raw constructor, the payload is left uninitialised
 * (malloc, not calloc): zero-filling 8 MB per getter call is work the MoonBit
 * runtime does not do, and it would be timed as part of the C4 read-back. */
moonbit_bytes_t moonbit_make_bytes_raw(int32_t len) {
  if (len < 0) len = 0;
  int32_t *h = (int32_t *)malloc(8 + (size_t)len + 1);
  if (!h) abort();
  h[0] = FAKE_RC;
  ((unsigned char *)(h + 2))[len] = 0;
  ((uint32_t *)h)[1] = (uint32_t)len & ((1u << 28) - 1);
  g_made++;
  return (moonbit_bytes_t)(h + 2);
}
/* the runtime's release of an object (the library drops a Bytes it built but
 * will not return, e.g. after a failed device copy, through this) */
void moonbit_decref(void *obj) {
  if (obj) free((int32_t *)obj - 2);
}
static int32_t mb_len(moonbit_bytes_t b) { return (int32_t)(((uint32_t *)b)[-1] & ((1u << 28) - 1)); }
static int32_t mb_rc(moonbit_bytes_t b) { return ((int32_t *)b)[-2]; }
static void mb_free(moonbit_bytes_t b) {
  if (b) free((int32_t *)b - 2);
}
static moonbit_bytes_t S(const char *s) {
  int32_t n = (int32_t)strlen(s);
  moonbit_bytes_t b = moonbit_make_bytes_raw(n);
  memcpy(b, s, (size_t)n);
  return b;
}

static int g_fail = 0;
#define CHECK(c, ...)                                \
  do {                                               \
    if (!(c)) {                                      \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                  \
      fprintf(stderr, "\n");                         \
      g_fail++;                                      \
    }                                                \
  } while (0)

/* a returned Bytes: check it came from this runtime, copy it out, release it */
static char *take(moonbit_bytes_t b) {
  static char buf[4096];
  if (!b) {
    buf[0] = 0;
    return buf;
  }
  CHECK(mb_rc(b) == FAKE_RC, "returned Bytes not allocated by the MoonBit runtime (rc=%d)", mb_rc(b));
  int32_t n = mb_len(b);
  if (n > (int32_t)sizeof(buf) - 1) n = sizeof(buf) - 1;
  memcpy(buf, b, (size_t)n);
  buf[n] = 0;
  mb_free(b);
  return buf;
}

static void check_cell(duckdb_mb_result *r, int col, int row, const char *want) {
  char *got = take(duckdb_mb_result_value(r, col, row));
  CHECK(strcmp(got, want) == 0, "cell(%d,%d) = '%s', want '%s'", col, row, got, want);
}

static duckdb_mb_connection *open_conn(int allow_no_gpu) {
  duckdb_mb_config *cfg = duckdb_mb_config_create();
  if (allow_no_gpu) {
    moonbit_bytes_t k = S("mbx_allow_no_gpu"), v = S("true");
    CHECK(duckdb_mb_config_set(cfg, k, v) == 1, "config_set mbx_allow_no_gpu");
    mb_free(k);
    mb_free(v);
  }
  moonbit_bytes_t bad_k = S("no_such_option"), bad_v = S("1");
  CHECK(duckdb_mb_config_set(cfg, bad_k, bad_v) == 0, "unknown config key must fail");
  CHECK(strstr(take(duckdb_mb_config_error(cfg)), "duckdb_set_config failed") != NULL, "config error text");
  mb_free(bad_k);
  mb_free(bad_v);
  moonbit_bytes_t path = S(":memory:");
  duckdb_mb_connection *c = duckdb_mb_connect_with_config(path, cfg);
  mb_free(path);
  duckdb_mb_config_destroy(cfg);
  CHECK(c && !duckdb_mb_is_null_conn(c), "connect: %s", take(duckdb_mb_last_error()));
  return c;
}

static void host_constant_checks(duckdb_mb_connection *c) {
  moonbit_bytes_t sql = S("SELECT 1 AS a, 'x' AS b, NULL AS n, 9223372036854775807 AS big, 5.0 / 2 AS d");
  duckdb_mb_result *r = duckdb_mb_query(c, sql);
  mb_free(sql);
  CHECK(r && !duckdb_mb_is_null_result(r), "query: %s", take(duckdb_mb_last_error()));
  if (!r) return;
  CHECK(duckdb_mb_result_column_count(r) == 5, "column_count");
  CHECK(duckdb_mb_result_row_count(r) == 1, "row_count");
  CHECK(strcmp(take(duckdb_mb_result_column_name(r, 1)), "b") == 0, "column_name");
  CHECK(duckdb_mb_result_column_type(r, 0) == 4, "INTEGER type id 4 (src/duckdb_parsing.mbt:8-52)");
  CHECK(duckdb_mb_result_column_type(r, 3) == 5, "BIGINT type id 5");
  CHECK(duckdb_mb_result_column_type(r, 4) == 11, "DOUBLE type id 11");
  check_cell(r, 0, 0, "1");
  check_cell(r, 1, 0, "x");
  CHECK(duckdb_mb_result_is_null(r, 2, 0) == 1, "is_null");
  check_cell(r, 3, 0, "9223372036854775807");
  check_cell(r, 4, 0, "2.5");
  duckdb_mb_result_destroy(r);

  /* errors: NULL result + message from duckdb_mb_last_error */
  sql = S("SELEC 1");
  r = duckdb_mb_query(c, sql);
  mb_free(sql);
  CHECK(r == NULL || duckdb_mb_is_null_result(r), "bad SQL must fail");
  CHECK(strlen(take(duckdb_mb_last_error())) > 0, "last_error set on failure");

  /* prepared statement with a bigint parameter (reference native test :210-227) */
  sql = S("SELECT ? * 2");
  duckdb_mb_statement *st = duckdb_mb_prepare(c, sql);
  mb_free(sql);
  CHECK(st && !duckdb_mb_is_null_statement(st), "prepare");
  if (st) {
    CHECK(duckdb_mb_bind_bigint(st, 1, 1000000000) == 1, "bind_bigint");
    r = duckdb_mb_execute_prepared(st);
    CHECK(r && !duckdb_mb_is_null_result(r), "execute_prepared");
    if (r) {
      check_cell(r, 0, 0, "2000000000");
      duckdb_mb_result_destroy(r);
    }
    duckdb_mb_statement_destroy(st);
  }
}

/* DataChunk / Vector / LogicalType handles without a device (ref :1944-2103) */
static void chunk_api_checks(void) {
  duckdb_mb_logical_type *bt = duckdb_mb_create_logical_type(5), *it = duckdb_mb_create_logical_type(4);
  CHECK(bt && it && !duckdb_mb_is_null_logical_type(bt), "create_logical_type");
  CHECK(duckdb_mb_is_null_logical_type(duckdb_mb_create_list_type(bt)), "LIST types are out of scope");
  CHECK(strstr(take(duckdb_mb_last_error()), "Not implemented") != NULL, "LIST error text");
  duckdb_logical_type types[2] = {bt->type, it->type};
  duckdb_mb_data_chunk *ch = duckdb_mb_create_data_chunk(types, 2);
  CHECK(ch && !duckdb_mb_is_null_data_chunk(ch), "create_data_chunk");
  duckdb_vector v0 = duckdb_mb_data_chunk_get_vector(ch, 0), v1 = duckdb_mb_data_chunk_get_vector(ch, 1);
  CHECK(v0 && v1 && duckdb_mb_data_chunk_get_vector(ch, 2) == NULL, "get_vector");
  uint64_t *val = duckdb_mb_vector_get_validity(v1);
  CHECK(val && val[0] == ~0ull && val[31] == ~0ull, "validity starts all-valid");
  val[0] &= ~1ull;
  duckdb_mb_data_chunk_reset(ch);
  CHECK(val[0] == ~0ull, "reset restores validity");
  CHECK(duckdb_mb_vector_get_data(v0) != NULL && duckdb_mb_list_vector_set_size(v0, 1) == DuckDBError, "vector data");
  duckdb_mb_destroy_data_chunk(ch);
  duckdb_mb_destroy_logical_type(bt);
  duckdb_mb_destroy_logical_type(it);
  CHECK(duckdb_mb_append_data_chunk(NULL, NULL) == 0, "append_data_chunk(NULL)");
}

/* two chunks into (v BIGINT, w INTEGER) with NULLs in both columns, then a
 * DECIMAL(18,3) chunk into a DECIMAL(15,2) column (converted value by value) */
static void chunk_append_checks(duckdb_mb_connection *c) {
  moonbit_bytes_t sql = S("CREATE TABLE dc (v BIGINT, w INTEGER, d DECIMAL(15,2))");
  duckdb_mb_result *r = duckdb_mb_query(c, sql);
  mb_free(sql);
  if (r) duckdb_mb_result_destroy(r);
  moonbit_bytes_t sch = S("main"), tab = S("dc");
  duckdb_mb_appender *ap = duckdb_mb_appender_create(c, sch, tab);
  mb_free(sch);
  mb_free(tab);
  CHECK(ap != NULL, "appender_create dc");
  if (!ap) return;
  duckdb_mb_logical_type *bt = duckdb_mb_create_logical_type(5), *it = duckdb_mb_create_logical_type(4),
                         *dt = duckdb_mb_create_logical_type(19);
  duckdb_logical_type types[3] = {bt->type, it->type, dt->type};
  duckdb_mb_data_chunk *ch = duckdb_mb_create_data_chunk(types, 3);
  for (int k = 0; k < 2; k++) {
    int64_t *v = duckdb_mb_vector_get_data(duckdb_mb_data_chunk_get_vector(ch, 0));
    int32_t *w = duckdb_mb_vector_get_data(duckdb_mb_data_chunk_get_vector(ch, 1));
    int64_t *d = duckdb_mb_vector_get_data(duckdb_mb_data_chunk_get_vector(ch, 2));
    uint64_t *vv = duckdb_mb_vector_get_validity(duckdb_mb_data_chunk_get_vector(ch, 0));
    uint64_t *wv = duckdb_mb_vector_get_validity(duckdb_mb_data_chunk_get_vector(ch, 1));
    for (int i = 0; i < 2048; i++) {
      v[i] = (int64_t)(k * 2048 + i) * 3;
      w[i] = k * 2048 + i;
      d[i] = 12345;  /* 12.345 at scale 3 -> 12.35 at scale 2 */
      if (i % 7 == 0) vv[i >> 6] &= ~(1ull << (i & 63));
      if (i % 11 == 0) wv[i >> 6] &= ~(1ull << (i & 63));
    }
    duckdb_mb_data_chunk_set_size(ch, 2048);
    CHECK(duckdb_mb_append_data_chunk(ap, ch) == 1, "append_data_chunk: %s", take(duckdb_mb_appender_error(ap)));
    duckdb_mb_data_chunk_reset(ch);
  }
  duckdb_mb_destroy_data_chunk(ch);
  duckdb_mb_destroy_logical_type(bt);
  duckdb_mb_destroy_logical_type(it);
  duckdb_mb_destroy_logical_type(dt);
  duckdb_mb_appender_destroy(ap); /* close => flush */
  sql = S("SELECT COUNT(*), COUNT(v), SUM(v), COUNT(w), SUM(w), MIN(d), MAX(d) FROM dc");
  r = duckdb_mb_query(c, sql);
  mb_free(sql);
  CHECK(r != NULL, "dc query: %s", take(duckdb_mb_last_error()));
  if (!r) return;
  long long cv = 0, sv = 0, cw = 0, sw = 0;
  for (int k = 0; k < 2; k++)
    for (int i = 0; i < 2048; i++) {
      if (i % 7) { cv++; sv += (long long)(k * 2048 + i) * 3; }
      if (i % 11) { cw++; sw += k * 2048 + i; }
    }
  char want[64];
  check_cell(r, 0, 0, "4096");
  snprintf(want, sizeof want, "%lld", cv); check_cell(r, 1, 0, want);
  snprintf(want, sizeof want, "%lld", sv); check_cell(r, 2, 0, want);
  snprintf(want, sizeof want, "%lld", cw); check_cell(r, 3, 0, want);
  snprintf(want, sizeof want, "%lld", sw); check_cell(r, 4, 0, want);
  check_cell(r, 5, 0, "12.35");
  check_cell(r, 6, 0, "12.35");
  duckdb_mb_result_destroy(r);
}

static int gpu_checks(duckdb_mb_connection *c, long rows) {
  char q[512];
  snprintf(q, sizeof q, "CREATE TABLE t AS SELECT mbx_synth(42, i, 50) + 1 AS x FROM range(%ld) tbl(i)", rows);
  moonbit_bytes_t sql = S(q);
  duckdb_mb_result *r = duckdb_mb_query(c, sql);
  mb_free(sql);
  CHECK(r != NULL, "CTAS: %s", take(duckdb_mb_last_error()));
  if (r) duckdb_mb_result_destroy(r);
  sql = S("SELECT COUNT(*) FROM t WHERE x > 24");
  r = duckdb_mb_query(c, sql);
  mb_free(sql);
  CHECK(r != NULL, "C2 query: %s", take(duckdb_mb_last_error()));
  if (r) {
    printf("count=%s\n", take(duckdb_mb_result_value(r, 0, 0)));
    duckdb_mb_result_destroy(r);
  }
  /* appender rows -> device -> Arrow int64 wire buffer [i32 count][int64 LE...] */
  sql = S("CREATE TABLE a (v BIGINT)");
  r = duckdb_mb_query(c, sql);
  mb_free(sql);
  if (r) duckdb_mb_result_destroy(r);
  moonbit_bytes_t sch = S("main"), tab = S("a");
  duckdb_mb_appender *ap = duckdb_mb_appender_create(c, sch, tab);
  mb_free(sch);
  mb_free(tab);
  CHECK(ap != NULL, "appender_create");
  for (int64_t i = 0; ap && i < 1000; i++) {
    duckdb_mb_begin_row(ap);
    duckdb_mb_append_bigint(ap, i * 2654435761LL);
    CHECK(duckdb_mb_end_row(ap) == 1, "end_row");
  }
  if (ap) duckdb_mb_appender_destroy(ap); /* close => flush */
  sql = S("SELECT v FROM a");
  duckdb_mb_arrow_result *ar = duckdb_mb_query_arrow(c, sql);
  mb_free(sql);
  CHECK(ar && !duckdb_mb_is_null_arrow_result(ar), "query_arrow");
  if (ar) {
    moonbit_bytes_t w = duckdb_mb_arrow_get_column_int64(ar, 0);
    CHECK(mb_rc(w) == FAKE_RC && mb_len(w) == 4 + 8 * 1000, "arrow int64 buffer size %d", mb_len(w));
    int32_t cnt;
    memcpy(&cnt, w, 4);
    CHECK(cnt == 1000, "arrow count %d", cnt);
    for (int i = 0; i < 1000; i++) {
      int64_t v;
      memcpy(&v, w + 4 + 8 * i, 8);
      if (v != (int64_t)i * 2654435761LL) {
        CHECK(0, "arrow value %d = %lld", i, (long long)v);
        break;
      }
    }
    mb_free(w);
    duckdb_mb_arrow_destroy(ar);
  }
  chunk_append_checks(c);
  return 0;
}

/* C4 through the reference's own row-wise Appender API, as a native MoonBit
 * caller drives it (src/duckdb_native.mbt:955-1076): 1 begin_row + 1
 * append_bigint + 1 end_row per row, close => flush; then the Arrow int64
 * getter over 1e6-row slices (the MoonBit decoder cap).  Values bit-exact.
 * Prints one JSON line. */

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}
static int64_t c4_value(int64_t i) { return (int64_t)(((uint64_t)i * 2654435761ull) & 0x7fffffffffffffffull); }

/* the chunked form of C4's ingest (ref duckdb_native.c:2029-2132): each
 * 2048-row BIGINT vector filled in place by one memcpy from the caller's
 * values (generated before the clock starts, as a MoonBit caller holds its
 * data), appended with duckdb_mb_append_data_chunk */
static int c4_ingest_chunks(duckdb_mb_appender *ap, const int64_t *src, long rows) {
  duckdb_mb_logical_type *bt = duckdb_mb_create_logical_type(5 /* DUCKDB_TYPE_BIGINT */);
  CHECK(!duckdb_mb_is_null_logical_type(bt), "create_logical_type");
  if (!bt) return 0;
  duckdb_logical_type types[1] = {bt->type};
  duckdb_mb_data_chunk *ch = duckdb_mb_create_data_chunk(types, 1);
  CHECK(!duckdb_mb_is_null_data_chunk(ch), "create_data_chunk");
  int ok = ch != NULL;
  for (long base = 0; ok && base < rows; base += 2048) {
    const long m = rows - base < 2048 ? rows - base : 2048;
    duckdb_vector v = duckdb_mb_data_chunk_get_vector(ch, 0);
    int64_t *d = (int64_t *)duckdb_mb_vector_get_data(v);
    memcpy(d, src + base, (size_t)m * 8);
    duckdb_mb_data_chunk_set_size(ch, (idx_t)m);
    ok &= duckdb_mb_append_data_chunk(ap, ch);
    duckdb_mb_data_chunk_reset(ch);
  }
  duckdb_mb_destroy_data_chunk(ch);
  duckdb_mb_destroy_logical_type(bt);
  return ok;
}

static int c4_bench(duckdb_mb_connection *c, long rows, int chunks) {
  moonbit_bytes_t sql = S("CREATE TABLE c4 (v BIGINT)");
  duckdb_mb_result *r = duckdb_mb_query(c, sql);
  mb_free(sql);
  if (r) duckdb_mb_result_destroy(r);
  /* untimed warm-up: the process's first large pageable H2D carries ~50 ms of
   * one-time runtime setup (profiles/r02_c4_probe.log) */
  sql = S("CREATE TABLE c4w (v BIGINT)");
  r = duckdb_mb_query(c, sql);
  mb_free(sql);
  if (r) duckdb_mb_result_destroy(r);
  /* the chunked ingest's source values, generated (and paged in) untimed */
  int64_t *src = NULL;
  if (chunks) {
    src = (int64_t *)malloc((size_t)rows * 8);
    CHECK(src != NULL, "c4 source array");
    if (!src) return 1;
    for (long i = 0; i < rows; i++) src[i] = c4_value(i);
  }
  moonbit_bytes_t sch = S("main"), tab = S("c4w");
  duckdb_mb_appender *ap = duckdb_mb_appender_create(c, sch, tab);
  mb_free(tab);
  if (ap) {
    if (chunks) {
      c4_ingest_chunks(ap, src, rows < 10000000 ? rows : 10000000);
    } else {
      for (int64_t i = 0; i < 3000000 && i < rows; i++) {
        duckdb_mb_begin_row(ap);
        duckdb_mb_append_bigint(ap, c4_value(i));
        duckdb_mb_end_row(ap);
      }
    }
    duckdb_mb_flush(ap);
    duckdb_mb_appender_destroy(ap);
  }
  sql = S("DROP TABLE c4w");
  r = duckdb_mb_query(c, sql);
  mb_free(sql);
  if (r) duckdb_mb_result_destroy(r);
  tab = S("c4");
  ap = duckdb_mb_appender_create(c, sch, tab);
  mb_free(sch);
  mb_free(tab);
  CHECK(ap != NULL, "appender_create");
  if (!ap) return 1;
  double t0 = now_s();
  int ok = 1;
  if (chunks) {
    ok &= c4_ingest_chunks(ap, src, rows);
  } else {
    for (int64_t i = 0; i < rows; i++) {
      ok &= duckdb_mb_begin_row(ap);
      ok &= duckdb_mb_append_bigint(ap, c4_value(i));
      ok &= duckdb_mb_end_row(ap);
    }
  }
  ok &= duckdb_mb_flush(ap);
  duckdb_mb_appender_destroy(ap);
  double t_in = now_s() - t0;
  /* the caller's own share of the chunked ingest: the same vector fills
   * (memcpy of each 2048-row vector into the chunk) without the appends */
  double t_fill = 0;
  if (chunks && src) {
    duckdb_mb_logical_type *bt = duckdb_mb_create_logical_type(5 /* DUCKDB_TYPE_BIGINT */);
    duckdb_logical_type types[1] = {bt->type};
    duckdb_mb_data_chunk *ch = duckdb_mb_create_data_chunk(types, 1);
    double f0 = now_s();
    for (long base = 0; base < rows; base += 2048) {
      const long m = rows - base < 2048 ? rows - base : 2048;
      int64_t *d = (int64_t *)duckdb_mb_vector_get_data(duckdb_mb_data_chunk_get_vector(ch, 0));
      memcpy(d, src + base, (size_t)m * 8);
      duckdb_mb_data_chunk_set_size(ch, (idx_t)m);
      duckdb_mb_data_chunk_reset(ch);
    }
    t_fill = now_s() - f0;
    duckdb_mb_destroy_data_chunk(ch);
    duckdb_mb_destroy_logical_type(bt);
  }
  free(src);
  CHECK(ok, "row-wise appends");
  /* untimed getter warm-up: the library's first 15 calls per size class are
   * its copy-method trials (hostlink.cpp MidLink); the timed loop below is the
   * steady state after them */
  for (long k = 0; k < rows && k < 20000000; k += 1000000) {
    char q[160];
    snprintf(q, sizeof q, "SELECT v FROM c4 LIMIT 1000000 OFFSET %ld", k);
    sql = S(q);
    duckdb_mb_arrow_result *ar = duckdb_mb_query_arrow(c, sql);
    mb_free(sql);
    if (!ar) break;
    moonbit_bytes_t w = duckdb_mb_arrow_get_column_int64(ar, 0);
    if (w) mb_free(w);
    duckdb_mb_arrow_destroy(ar);
  }
  /* query_arrow + getter timed; the value check of each Bytes is outside the clock */
  double t_out = 0, t_qa = 0;
  long checked = 0, bad = 0;
  for (long k = 0; k < rows; k += 1000000) {
    char q[160];
    snprintf(q, sizeof q, "SELECT v FROM c4 LIMIT 1000000 OFFSET %ld", k);
    sql = S(q);
    t0 = now_s();
    duckdb_mb_arrow_result *ar = duckdb_mb_query_arrow(c, sql);
    t_qa += now_s() - t0;
    moonbit_bytes_t w = ar ? duckdb_mb_arrow_get_column_int64(ar, 0) : NULL;
    t_out += now_s() - t0;
    mb_free(sql);
    if (!ar) { bad++; break; }
    int32_t cnt;
    memcpy(&cnt, w, 4);
    for (int32_t i = 0; i < cnt; i++) {
      int64_t v;
      memcpy(&v, w + 4 + 8 * (size_t)i, 8);
      bad += v != c4_value(k + i);
    }
    checked += cnt;
    mb_free(w);
    duckdb_mb_arrow_destroy(ar);
  }
  CHECK(checked == rows && bad == 0, "c4 read-back: %ld rows checked, %ld mismatches", checked, bad);
  /* the query_stream leg (ref duckdb_native.mbt:504-582: per-cell strings of
   * <= 2048-row chunks) over a bounded prefix: every cell pulled and parsed as
   * the MoonBit driver would, each value checked */
  const long srows = rows < 10000000 ? rows : 10000000;
  char q[160];
  snprintf(q, sizeof q, "SELECT v FROM c4 LIMIT %ld", srows);
  sql = S(q);
  t0 = now_s();
  duckdb_mb_stream *st = duckdb_mb_query_stream(c, sql);
  mb_free(sql);
  CHECK(st != NULL, "c4 stream: %s", take(duckdb_mb_last_error()));
  long sgot = 0, sbad = 0;
  while (st) {
    duckdb_mb_chunk *ch = duckdb_mb_stream_fetch_chunk(st);
    if (!ch) break;
    const int32_t nr = duckdb_mb_chunk_row_count(ch);
    for (int32_t i = 0; i < nr; i++) {
      moonbit_bytes_t v = duckdb_mb_chunk_value(ch, 0, i);
      char buf[32];
      const int32_t n = mb_len(v) < 31 ? mb_len(v) : 31;
      memcpy(buf, v, (size_t)n);
      buf[n] = 0;
      sbad += strtoll(buf, NULL, 10) != c4_value(sgot + i);
      mb_free(v);
    }
    sgot += nr;
    duckdb_mb_chunk_destroy(ch);
  }
  if (st) duckdb_mb_stream_destroy(st);
  const double t_st = now_s() - t0;
  CHECK(sgot == srows && sbad == 0, "c4 stream: %ld rows, %ld mismatches", sgot, sbad);
  char *link = duckdb_mbx_link_stats();
  printf("{\"link_mid_stats\": %s, ", link ? link : "null");
  duckdb_mbx_free(link);
  if (chunks)
    printf("\"caller_fill_s\": %.6f, \"caller_fill_gbs\": %.3f, \"library_s\": %.6f, \"library_gbs\": %.3f, ", t_fill,
           rows * 8.0 / t_fill / 1e9, t_in - t_fill, rows * 8.0 / (t_in - t_fill) / 1e9);
  printf("\"rows\": %ld, \"ingest_api\": \"%s\", \"ingest_s\": %.6f, \"ingest_rows_per_s\": %.1f, "
         "\"ingest_gbs\": %.3f, \"readback_s\": %.6f, \"readback_gbs\": %.3f, \"readback_query_s\": %.6f, "
         "\"readback_getter_gbs\": %.3f, \"stream_rows\": %ld, "
         "\"stream_s\": %.6f, \"stream_rows_per_s\": %.1f, \"bit_exact\": %s}\n",
         rows, chunks ? "append_data_chunk" : "begin_row/append_bigint/end_row", t_in, rows / t_in,
         rows * 8.0 / t_in / 1e9, t_out, rows * 8.0 / t_out / 1e9, t_qa, rows * 8.0 / (t_out - t_qa) / 1e9, sgot,
         t_st, sgot / t_st,
         (checked == rows && bad == 0 && sgot == srows && sbad == 0) ? "true" : "false");
  return 0;
}

/* C1 (BASELINE configs[0]): SELECT i FROM range(1000000) WHERE i%2=0 the way
 * the MoonBit driver consumes it — Connection::query's per-cell pull
 * (duckdb_native.mbt:454-501: is_null + value per cell) and query_stream's
 * chunk loop (:504-582) — checking 500 000 rows and their sum
 * 249 999 500 000.  Prints one JSON line (best of `reps`). */
static int c1_bench(duckdb_mb_connection *c, int reps) {
  const char *q = "SELECT i FROM range(1000000) tbl(i) WHERE i%2=0";
  double best_q = 1e30, best_s = 1e30, best_exec = 1e30, best_first = 1e30;
  long long sum_q = 0, sum_s = 0;
  long rows_q = 0, rows_s = 0, chunks = 0;
  for (int rep = 0; rep < reps; rep++) {
    double t0 = now_s();
    moonbit_bytes_t sql = S(q);
    duckdb_mb_result *r = duckdb_mb_query(c, sql);
    mb_free(sql);
    CHECK(r != NULL, "c1 query: %s", take(duckdb_mb_last_error()));
    if (!r) return 1;
    const double te = now_s() - t0;
    if (te < best_exec) best_exec = te;
    rows_q = duckdb_mb_result_row_count(r);
    sum_q = 0;
    for (int32_t i = 0; i < rows_q; i++) {
      if (duckdb_mb_result_is_null(r, 0, i)) continue;
      moonbit_bytes_t v = duckdb_mb_result_value(r, 0, i);
      char buf[32];
      int32_t n = mb_len(v) < 31 ? mb_len(v) : 31;
      memcpy(buf, v, (size_t)n);
      buf[n] = 0;
      sum_q += atoll(buf);
      mb_free(v);
    }
    duckdb_mb_result_destroy(r);
    double t1 = now_s();
    if (t1 - t0 < best_q) best_q = t1 - t0;
    sql = S(q);
    duckdb_mb_stream *st = duckdb_mb_query_stream(c, sql);
    mb_free(sql);
    CHECK(st != NULL, "c1 stream: %s", take(duckdb_mb_last_error()));
    if (!st) return 1;
    rows_s = 0;
    sum_s = 0;
    chunks = 0;
    for (;;) {
      duckdb_mb_chunk *ch = duckdb_mb_stream_fetch_chunk(st);
      if (!ch) break;
      if (chunks == 0 && now_s() - t1 < best_first) best_first = now_s() - t1;
      int32_t nr = duckdb_mb_chunk_row_count(ch);
      for (int32_t i = 0; i < nr; i++) {
        moonbit_bytes_t v = duckdb_mb_chunk_value(ch, 0, i);
        char buf[32];
        int32_t n = mb_len(v) < 31 ? mb_len(v) : 31;
        memcpy(buf, v, (size_t)n);
        buf[n] = 0;
        sum_s += atoll(buf);
        mb_free(v);
      }
      rows_s += nr;
      chunks++;
      duckdb_mb_chunk_destroy(ch);
    }
    CHECK(strlen(take(duckdb_mb_last_error())) == 0, "end of stream must leave an empty error");
    duckdb_mb_stream_destroy(st);
    double t2 = now_s();
    if (t2 - t1 < best_s) best_s = t2 - t1;
  }
  const int ok = rows_q == 500000 && sum_q == 249999500000LL && rows_s == 500000 && sum_s == 249999500000LL;
  CHECK(ok, "c1: query %ld rows sum %lld, stream %ld rows sum %lld", rows_q, sum_q, rows_s, sum_s);
  printf("{\"rows\": %ld, \"query_percell_s\": %.6f, \"query_rows_per_s\": %.1f, \"query_exec_s\": %.6f, "
         "\"stream_s\": %.6f, \"stream_rows_per_s\": %.1f, \"stream_first_chunk_s\": %.6f, \"stream_chunks\": %ld, "
         "\"sum\": %lld, \"exact\": %s}\n",
         rows_q, best_q, rows_q / best_q, best_exec, best_s, rows_s / best_s, best_first, chunks, sum_q,
         ok ? "true" : "false");
  return 0;
}

/* every line of a file is one statement: run it, read every cell of a result
 * (errors are expected for statements that need a device); used to drive the
 * parser / binder / formatter under AddressSanitizer + UBSan */
static int sql_file(duckdb_mb_connection *c, const char *path) {
  FILE *f = fopen(path, "r");
  CHECK(f != NULL, "open %s", path);
  if (!f) return 1;
  static char line[1 << 16];
  long ok = 0, failed = 0;
  while (fgets(line, sizeof line, f)) {
    size_t n = strlen(line);
    while (n && (line[n - 1] == '\n' || line[n - 1] == '\r')) line[--n] = 0;
    if (!n) continue;
    moonbit_bytes_t sql = S(line);
    duckdb_mb_result *r = duckdb_mb_query(c, sql);
    if (r) {
      const int32_t nc = duckdb_mb_result_column_count(r), nr = duckdb_mb_result_row_count(r);
      for (int32_t j = 0; j < nc; j++) {
        (void)take(duckdb_mb_result_column_name(r, j));
        (void)duckdb_mb_result_column_type(r, j);
        for (int32_t i = 0; i < nr; i++) {
          (void)duckdb_mb_result_is_null(r, j, i);
          (void)take(duckdb_mb_result_value(r, j, i));
        }
      }
      duckdb_mb_result_destroy(r);
      ok++;
    } else {
      (void)take(duckdb_mb_last_error());
      failed++;
    }
    /* the same text as a prepared statement and a stream */
    duckdb_mb_statement *st = duckdb_mb_prepare(c, sql);
    if (st) {
      duckdb_mb_result *pr = duckdb_mb_execute_prepared(st);
      if (pr) duckdb_mb_result_destroy(pr);
      duckdb_mb_statement_destroy(st);
    }
    mb_free(sql);
  }
  fclose(f);
  printf("sqlfile: %ld ok, %ld failed\n", ok, failed);
  return 0;
}

int main(int argc, char **argv) {
  const char *mode = argc > 1 ? argv[1] : "cpu";
  if (strcmp(mode, "sqlfile") == 0) {
    duckdb_mb_connection *c = open_conn(1);
    if (!c) return 1;
    sql_file(c, argc > 2 ? argv[2] : "/dev/null");
    duckdb_mb_disconnect(c);
    return g_fail ? 1 : 0;
  }
  int gpu = strcmp(mode, "gpu") == 0, c4 = strcmp(mode, "c4") == 0, c1 = strcmp(mode, "c1") == 0;
  const int c4chunk = strcmp(mode, "c4chunk") == 0;
  c4 |= c4chunk;
  duckdb_mb_connection *c = open_conn(!gpu && !c4 && !c1);
  if (!c) return 1;
  if (c1) {
    c1_bench(c, argc > 2 ? atoi(argv[2]) : 5);
    duckdb_mb_disconnect(c);
    return g_fail ? 1 : 0;
  }
  if (c4) {
    c4_bench(c, argc > 2 ? atol(argv[2]) : 100000000, c4chunk);
    duckdb_mb_disconnect(c);
    return g_fail ? 1 : 0;
  }
  host_constant_checks(c);
  chunk_api_checks();
  if (gpu) gpu_checks(c, argc > 2 ? atol(argv[2]) : 1000000);
  duckdb_mb_disconnect(c);
  CHECK(g_made > 0, "no Bytes made through the runtime allocator");
  printf("harness %s: %s (%ld runtime Bytes)\n", mode, g_fail ? "FAILED" : "ok", g_made);
  return g_fail ? 1 : 0;
}
