/*
 * duckdb_mb.h — the drop-in C-ABI boundary of the MI355X columnar backend.
 *
 * These are exactly the 89 `duckdb_mb_*` symbols the reference's MoonBit
 * driver binds with `extern "C" fn ... = "duckdb_mb_*"`:
 *   72 in /root/reference/src/duckdb_native.mbt:10-411, :669-743
 *   17 in /root/reference/src/duckdb_arrow_native.mbt:10-104
 * with the C parameter/return types of their definitions in
 * /root/reference/src/duckdb_native.c (the line cited on each declaration is
 * the reference definition this symbol replaces).  The library
 * `libduckdb_mb_amd.so` (built from duckdb.mbt_amd/csrc) exports all of them;
 * it links no libduckdb.  Scans, filters, projections and aggregates run as
 * hand-written gfx950 HIP kernels on device-resident column chunks.
 *
 * ABI rules kept from the reference (refs/ffi.md:258-281, :509-547):
 *   - MoonBit Int/Bool -> int32_t, Int64 -> int64_t, Double -> double,
 *     Bytes -> uint8_t* with the MoonBit object header in front (the length is
 *     read with Moonbit_array_length), Array[Bytes] -> uint8_t**.
 *   - every pointer argument is borrowed; returned Bytes are fresh objects from
 *     moonbit_make_bytes_raw owned by the caller.
 *   - failure = NULL handle or 0 status; the message comes from
 *     duckdb_mb_last_error() (connect/query/stream/arrow) or the per-handle
 *     *_error() accessor (statement/appender/config).
 *   - end of stream = NULL chunk with an EMPTY last error
 *     (reference duckdb_native.c:466-490).
 *
 * Extensions (prefix duckdb_mbx_, not part of the reference surface) are
 * declared at the bottom: helpers for non-MoonBit hosts (Python/ctypes tests)
 * and the columnar bulk-ingest / profiling entry points.
 */
#ifndef DUCKDB_MB_AMD_H
#define DUCKDB_MB_AMD_H

#include <stdbool.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef uint8_t *moonbit_bytes_t;

/* Opaque handles (the MoonBit side sees them as #external = void*). */
typedef struct duckdb_mb_connection duckdb_mb_connection;
typedef struct duckdb_mb_result duckdb_mb_result; /* reference: duckdb_result* */
typedef struct duckdb_mb_stream duckdb_mb_stream;
typedef struct duckdb_mb_chunk duckdb_mb_chunk;
typedef struct duckdb_mb_statement duckdb_mb_statement;
typedef struct duckdb_mb_appender duckdb_mb_appender;
typedef struct duckdb_mb_config duckdb_mb_config;
typedef struct duckdb_mb_arrow_result duckdb_mb_arrow_result;

/* ---- connection (duckdb_native.c:67-140, :248-250) ---------------------- */
duckdb_mb_connection *duckdb_mb_connect(moonbit_bytes_t path);                  /* :67   */
void duckdb_mb_disconnect(duckdb_mb_connection *handle);                         /* :133  */
int32_t duckdb_mb_is_null_conn(duckdb_mb_connection *handle);                    /* :248  */
moonbit_bytes_t duckdb_mb_last_error(void);                                      /* :240  */

/* ---- materialized query (duckdb_native.c:142-254) ---------------------- */
duckdb_mb_result *duckdb_mb_query(duckdb_mb_connection *handle, moonbit_bytes_t sql); /* :142 */
void duckdb_mb_result_destroy(duckdb_mb_result *result);                         /* :174  */
int32_t duckdb_mb_result_column_count(duckdb_mb_result *result);                 /* :182  */
int32_t duckdb_mb_result_row_count(duckdb_mb_result *result);                    /* :189  */
moonbit_bytes_t duckdb_mb_result_column_name(duckdb_mb_result *result, int32_t col); /* :196 */
int32_t duckdb_mb_result_column_type(duckdb_mb_result *result, int32_t col);     /* :208  */
int32_t duckdb_mb_result_is_null(duckdb_mb_result *result, int32_t col, int32_t row); /* :215 */
moonbit_bytes_t duckdb_mb_result_value(duckdb_mb_result *result, int32_t col, int32_t row); /* :224 */
int32_t duckdb_mb_is_null_result(duckdb_mb_result *result);                      /* :252  */

/* ---- streaming (duckdb_native.c:260-667) ------------------------------- */
duckdb_mb_stream *duckdb_mb_query_stream(duckdb_mb_connection *handle, moonbit_bytes_t sql); /* :355 */
duckdb_mb_stream *duckdb_mb_execute_prepared_stream(duckdb_mb_statement *stmt);  /* :399  */
void duckdb_mb_stream_destroy(duckdb_mb_stream *stream);                         /* :426  */
int32_t duckdb_mb_is_null_stream(duckdb_mb_stream *stream);                      /* :440  */
int32_t duckdb_mb_stream_column_count(duckdb_mb_stream *stream);                 /* :444  */
moonbit_bytes_t duckdb_mb_stream_column_name(duckdb_mb_stream *stream, int32_t col); /* :451 */
duckdb_mb_chunk *duckdb_mb_stream_fetch_chunk(duckdb_mb_stream *stream);         /* :466  */
void duckdb_mb_chunk_destroy(duckdb_mb_chunk *chunk);                            /* :492  */
int32_t duckdb_mb_is_null_chunk(duckdb_mb_chunk *chunk);                         /* :502  */
int32_t duckdb_mb_chunk_row_count(duckdb_mb_chunk *chunk);                       /* :506  */
int32_t duckdb_mb_chunk_column_count(duckdb_mb_chunk *chunk);                    /* :513  */
int32_t duckdb_mb_chunk_is_null(duckdb_mb_chunk *chunk, int32_t col, int32_t row); /* :520 */
moonbit_bytes_t duckdb_mb_chunk_value(duckdb_mb_chunk *chunk, int32_t col, int32_t row); /* :537 */

/* ---- configuration (duckdb_native.c:673-810) --------------------------- */
duckdb_mb_config *duckdb_mb_config_create(void);                                 /* :678  */
void duckdb_mb_config_destroy(duckdb_mb_config *cfg);                            /* :697  */
moonbit_bytes_t duckdb_mb_config_error(duckdb_mb_config *cfg);                   /* :707  */
int32_t duckdb_mb_config_set(duckdb_mb_config *cfg, moonbit_bytes_t key, moonbit_bytes_t value); /* :714 */
duckdb_mb_connection *duckdb_mb_connect_with_config(moonbit_bytes_t path, duckdb_mb_config *cfg); /* :749 */

/* ---- prepared statements (duckdb_native.c:816-1020, :1261-1296) -------- */
duckdb_mb_statement *duckdb_mb_prepare(duckdb_mb_connection *handle, moonbit_bytes_t sql); /* :816 */
void duckdb_mb_statement_destroy(duckdb_mb_statement *stmt);                     /* :856  */
moonbit_bytes_t duckdb_mb_statement_error(duckdb_mb_statement *stmt);            /* :866  */
int32_t duckdb_mb_bind_int(duckdb_mb_statement *stmt, int32_t index, int32_t value);   /* :873  */
int32_t duckdb_mb_bind_bigint(duckdb_mb_statement *stmt, int32_t index, int64_t value); /* :890 */
int32_t duckdb_mb_bind_double(duckdb_mb_statement *stmt, int32_t index, double value);  /* :907 */
int32_t duckdb_mb_bind_varchar(duckdb_mb_statement *stmt, int32_t index, moonbit_bytes_t value); /* :924 */
int32_t duckdb_mb_bind_bool(duckdb_mb_statement *stmt, int32_t index, bool value);      /* :950 */
int32_t duckdb_mb_bind_null(duckdb_mb_statement *stmt, int32_t index);           /* :967  */
int32_t duckdb_mb_clear_bindings(duckdb_mb_statement *stmt);                     /* :983  */
duckdb_mb_result *duckdb_mb_execute_prepared(duckdb_mb_statement *stmt);         /* :991  */
int32_t duckdb_mb_is_null_statement(duckdb_mb_statement *stmt);                  /* :1018 */
int32_t duckdb_mb_bind_date(duckdb_mb_statement *stmt, int32_t index, int32_t days);    /* :1261 */
int32_t duckdb_mb_bind_timestamp(duckdb_mb_statement *stmt, int32_t index, int64_t micros); /* :1279 */
int32_t duckdb_mb_bind_blob(duckdb_mb_statement *stmt, int32_t index, moonbit_bytes_t data, int32_t length); /* :1377 */
int32_t duckdb_mb_bind_decimal(duckdb_mb_statement *stmt, int32_t index, uint8_t width, uint8_t scale,
                               int64_t lower, int64_t upper);                    /* :1421 */
int32_t duckdb_mb_bind_interval(duckdb_mb_statement *stmt, int32_t index, int32_t months, int32_t days,
                                int64_t micros);                                 /* :1487 */
int32_t duckdb_mb_bind_list_varchar(duckdb_mb_statement *stmt, int32_t index, moonbit_bytes_t *values,
                                    int32_t count);                              /* :1539 */
int32_t duckdb_mb_bind_struct_varchar(duckdb_mb_statement *stmt, int32_t index, moonbit_bytes_t *field_names,
                                      moonbit_bytes_t *field_values, int32_t field_count); /* :1597 */
int32_t duckdb_mb_bind_map_varchar_varchar(duckdb_mb_statement *stmt, int32_t index, moonbit_bytes_t *keys,
                                           moonbit_bytes_t *values, int32_t entry_count); /* :1666 */

/* ---- appender (duckdb_native.c:1026-1255, :1313-1367, :1397-1533, :1735-1922) */
duckdb_mb_appender *duckdb_mb_appender_create(duckdb_mb_connection *handle, moonbit_bytes_t schema,
                                              moonbit_bytes_t table);            /* :1032 */
void duckdb_mb_appender_destroy(duckdb_mb_appender *app);                        /* :1083 */
moonbit_bytes_t duckdb_mb_appender_error(duckdb_mb_appender *app);               /* :1093 */
int32_t duckdb_mb_begin_row(duckdb_mb_appender *app);                            /* :1100 */
int32_t duckdb_mb_append_int(duckdb_mb_appender *app, int32_t value);            /* :1116 */
int32_t duckdb_mb_append_bigint(duckdb_mb_appender *app, int64_t value);         /* :1132 */
int32_t duckdb_mb_append_double(duckdb_mb_appender *app, double value);          /* :1148 */
int32_t duckdb_mb_append_varchar(duckdb_mb_appender *app, moonbit_bytes_t value); /* :1164 */
int32_t duckdb_mb_append_bool(duckdb_mb_appender *app, bool value);              /* :1189 */
int32_t duckdb_mb_append_null(duckdb_mb_appender *app);                          /* :1205 */
int32_t duckdb_mb_end_row(duckdb_mb_appender *app);                              /* :1221 */
int32_t duckdb_mb_flush(duckdb_mb_appender *app);                                /* :1237 */
int32_t duckdb_mb_is_null_appender(duckdb_mb_appender *app);                     /* :1253 */
int32_t duckdb_mb_append_date(duckdb_mb_appender *app, int32_t days);            /* :1313 */
int32_t duckdb_mb_append_timestamp(duckdb_mb_appender *app, int64_t micros);     /* :1350 */
int32_t duckdb_mb_append_blob(duckdb_mb_appender *app, moonbit_bytes_t data, int32_t length); /* :1397 */
int32_t duckdb_mb_append_decimal(duckdb_mb_appender *app, uint8_t width, uint8_t scale, int64_t lower,
                                 int64_t upper);                                 /* :1447 */
int32_t duckdb_mb_append_interval(duckdb_mb_appender *app, int32_t months, int32_t days, int64_t micros); /* :1511 */
int32_t duckdb_mb_append_list_varchar(duckdb_mb_appender *app, moonbit_bytes_t *values, int32_t count); /* :1735 */
int32_t duckdb_mb_append_struct_varchar(duckdb_mb_appender *app, moonbit_bytes_t *field_names,
                                        moonbit_bytes_t *field_values, int32_t field_count); /* :1792 */
int32_t duckdb_mb_append_map_varchar_varchar(duckdb_mb_appender *app, moonbit_bytes_t *keys,
                                             moonbit_bytes_t *values, int32_t entry_count); /* :1860 */

/* ---- "arrow" columnar read-back (duckdb_native.c:2211-2797) ------------ */
duckdb_mb_arrow_result *duckdb_mb_query_arrow(duckdb_mb_connection *handle, moonbit_bytes_t sql); /* :2219 */
void duckdb_mb_arrow_destroy(duckdb_mb_arrow_result *r);                         /* :2548 */
int32_t duckdb_mb_arrow_column_count(duckdb_mb_arrow_result *r);                 /* :2270 */
int32_t duckdb_mb_arrow_row_count(duckdb_mb_arrow_result *r);                    /* :2277 */
moonbit_bytes_t duckdb_mb_arrow_schema(duckdb_mb_arrow_result *r);               /* :2285 */
moonbit_bytes_t duckdb_mb_arrow_get_column_int32(duckdb_mb_arrow_result *r, int32_t col);  /* :2359 */
moonbit_bytes_t duckdb_mb_arrow_get_column_int64(duckdb_mb_arrow_result *r, int32_t col);  /* :2392 */
moonbit_bytes_t duckdb_mb_arrow_get_column_double(duckdb_mb_arrow_result *r, int32_t col); /* :2424 */
moonbit_bytes_t duckdb_mb_arrow_get_column_string(duckdb_mb_arrow_result *r, int32_t col); /* :2456 */
moonbit_bytes_t duckdb_mb_arrow_get_column_bool(duckdb_mb_arrow_result *r, int32_t col);   /* :2516 */
moonbit_bytes_t duckdb_mb_arrow_get_column_int32_nullable(duckdb_mb_arrow_result *r, int32_t col);  /* :2572 */
moonbit_bytes_t duckdb_mb_arrow_get_column_int64_nullable(duckdb_mb_arrow_result *r, int32_t col);  /* :2611 */
moonbit_bytes_t duckdb_mb_arrow_get_column_double_nullable(duckdb_mb_arrow_result *r, int32_t col); /* :2649 */
moonbit_bytes_t duckdb_mb_arrow_get_column_string_nullable(duckdb_mb_arrow_result *r, int32_t col); /* :2687 */
moonbit_bytes_t duckdb_mb_arrow_get_column_bool_nullable(duckdb_mb_arrow_result *r, int32_t col);   /* :2761 */
int32_t duckdb_mb_is_null_arrow_result(duckdb_mb_arrow_result *r);               /* :2556 */
double duckdb_mb_bytes_to_double(const char *bytes, int32_t offset);             /* :2561 */

/* ======================================================================== *
 * Extensions (not in the reference surface).                                *
 * ======================================================================== */

/* MoonBit byte objects for hosts that are not a MoonBit program.  Inside a
 * MoonBit executable the runtime's moonbit_make_bytes_raw and moonbit_decref
 * are used instead (ours are weak definitions); the
 * library calls moonbit_decref only on a Bytes it built and does not return. */
moonbit_bytes_t moonbit_make_bytes_raw(int32_t len);
void moonbit_decref(void *obj);
moonbit_bytes_t duckdb_mbx_bytes_new(const uint8_t *data, int32_t len);
int32_t duckdb_mbx_bytes_len(moonbit_bytes_t bytes);
void duckdb_mbx_bytes_free(moonbit_bytes_t bytes);

/* Device / library info: number of visible gfx950 devices (0 without a GPU),
 * and the library build string. */
int32_t duckdb_mbx_device_count(void);
const char *duckdb_mbx_version(void);

/* Plan of a statement as text (binder + planner only, never touches a GPU).
 * Returns a malloc'd NUL-terminated string (free with duckdb_mbx_free) or NULL
 * with duckdb_mb_last_error() set. */
char *duckdb_mbx_explain(duckdb_mb_connection *handle, const char *sql, int64_t sql_len);
void duckdb_mbx_free(void *p);
/* Run-time compiled expression kernels (hipRTC, gfx950): compiles the kernels
 * of a fixed sample program without a GPU; NULL = ok, else the compiler log
 * (free with duckdb_mbx_free). */
char *duckdb_mbx_jit_selftest(void);
/* Waits for pending background kernel compiles (also done by
 * duckdb_mb_disconnect).  Hosts that exit without disconnecting call it
 * first: exit() must not tear the compiler down under a running compile. */
void duckdb_mbx_jit_join(void);

/* Columnar bulk ingest (MI355X-native form of the unbound
 * duckdb_mb_append_data_chunk, reference duckdb_native.c:2109-2132):
 * appends `count` values of one column from host memory; all columns of a
 * batch must be appended with the same count before duckdb_mbx_append_commit.
 * `validity` may be NULL (all valid) or one byte per row (1 = valid). */
int32_t duckdb_mbx_append_column(duckdb_mb_appender *app, int32_t col, const void *values,
                                 const uint8_t *validity, int64_t count);
int32_t duckdb_mbx_append_commit(duckdb_mb_appender *app, int64_t count);

/* Per-query device profile of the last statement run on this connection
 * (enable with config key "mbx_profile"="true"): JSON text, malloc'd. */
char *duckdb_mbx_last_profile(duckdb_mb_connection *handle);
/* Every kernel timing recorded since the previous drain (JSON array), then clears. */
char *duckdb_mbx_profile_drain(duckdb_mb_connection *handle);

/* HBM calibration on the connection's device: best-of-`iters` GB/s of a
 * float4 copy (read+write bytes), a non-temporal int64 read and a plain int64
 * read over `bytes`-sized buffers -> out3[0..2].  Returns 1 on success. */
int32_t duckdb_mbx_hbm_calibrate(duckdb_mb_connection *handle, int64_t bytes, int32_t iters, double *out3);
/* the same plus the hot kernels' shapes: out[0..7] = copy, nt read, read,
 * LDS-DMA ring read, unrolled nt copy, LDS-DMA ring copy, ring copy writing
 * half of what it reads, C3's two-array ring read (4-byte + 8-byte column,
 * 2-deep 3 KiB slots) (GB/s; a copy counts read + write); returns how many
 * were written (<= nout), 0 on error */
int32_t duckdb_mbx_hbm_calibrate_ex(duckdb_mb_connection *handle, int64_t bytes, int32_t iters, double *out,
                                    int32_t nout);
/* Arrow getter copies of 2-32 MiB (ref src/duckdb_native.c:2392-2422 fills
 * an 8 MB Bytes per 1e6-row INT64 slice): by default, per device and size
 * class, the first calls try the runtime's copy, a registered destination
 * and a pinned bounce (5 calls each) and the class keeps the fastest median.
 * duckdb_mbx_set_link_mode pins one method process-wide from now on (-1 the
 * measured choice, 0 runtime, 1 register, 2 bounce; returns 1);
 * duckdb_mbx_link_stats reports each class's trial medians (GB/s), the method
 * kept and the calls served, as JSON (free with duckdb_mbx_free). */
int32_t duckdb_mbx_set_link_mode(int32_t mode);
char *duckdb_mbx_link_stats(void);
/* Diagnostic build only (`make -C duckdb.mbt_amd clockdiag` ->
 * libduckdb_mb_amd_clk.so): the in-kernel clock stamps of the last
 * filter_agg_lds / group_direct_lds / two-array ring launch, 4 values per
 * workgroup {s_memtime, s_memrealtime at the main loop's start, the same at
 * its end}; clock = d(memtime) / d(realtime) x 100 MHz.  Returns the
 * workgroups copied (<= cap); 0 from the product library, which has no stamps. */
int32_t duckdb_mbx_clock_stamps(duckdb_mb_connection *handle, uint64_t *out4, int32_t cap);

/* ---- DataChunk / Vector / LogicalType (ref src/duckdb_native.c:1926-2132) ----
 * The reference wraps libduckdb's data-chunk API; these handles keep its C
 * signatures (duckdb.h handle and enum types declared below) over host-side
 * vectors of DuckDB's vector size (2048 rows).  duckdb_mb_append_data_chunk
 * copies a chunk's fixed-width vectors into the appender's pinned double
 * buffer (whole-vector copies; the buffer's async H2D DMA as for the row-wise
 * appender).  LIST/STRUCT/MAP types and list vectors are out of scope
 * (NULL / DuckDBError with "Not implemented"). */
#ifndef DUCKDB_API_HANDLES_DECLARED
#define DUCKDB_API_HANDLES_DECLARED
typedef uint64_t idx_t;
typedef enum duckdb_state { DuckDBSuccess = 0, DuckDBError = 1 } duckdb_state;
typedef int32_t duckdb_type; /* DUCKDB_TYPE_* ids: BOOLEAN 1 ... BIGINT 5 ... DOUBLE 11 ... HUGEINT 16, DECIMAL 19 */
typedef struct _duckdb_logical_type { void *internal_ptr; } * duckdb_logical_type;
typedef struct _duckdb_vector { void *internal_ptr; } * duckdb_vector;
typedef struct _duckdb_data_chunk { void *internal_ptr; } * duckdb_data_chunk;
#endif
typedef struct duckdb_mb_logical_type { duckdb_logical_type type; } duckdb_mb_logical_type; /* ref :1928-1930 */
typedef struct duckdb_mb_data_chunk { duckdb_data_chunk chunk; } duckdb_mb_data_chunk;     /* ref :1932-1934 */

duckdb_mb_logical_type *duckdb_mb_create_logical_type(duckdb_type type_id);            /* ref :1944-1956 */
duckdb_mb_logical_type *duckdb_mb_create_list_type(duckdb_mb_logical_type *child_type); /* ref :1958-1973 */
duckdb_mb_logical_type *duckdb_mb_create_struct_type(duckdb_logical_type *member_types, const char **member_names,
                                                     idx_t member_count);               /* ref :1975-1990 */
duckdb_mb_logical_type *duckdb_mb_create_map_type(duckdb_logical_type *key_type,
                                                  duckdb_logical_type *value_type);     /* ref :1992-2009 */
void duckdb_mb_destroy_logical_type(duckdb_mb_logical_type *mb_type);                   /* ref :2011-2019 */
int32_t duckdb_mb_is_null_logical_type(duckdb_mb_logical_type *mb_type);               /* ref :2021-2023 */
duckdb_mb_data_chunk *duckdb_mb_create_data_chunk(duckdb_logical_type *types, idx_t column_count); /* ref :2029-2043 */
void duckdb_mb_destroy_data_chunk(duckdb_mb_data_chunk *mb_chunk);                      /* ref :2045-2053 */
duckdb_vector duckdb_mb_data_chunk_get_vector(duckdb_mb_data_chunk *mb_chunk, idx_t col_idx); /* ref :2055-2061 */
void duckdb_mb_data_chunk_set_size(duckdb_mb_data_chunk *mb_chunk, idx_t size);        /* ref :2063-2068 */
void duckdb_mb_data_chunk_reset(duckdb_mb_data_chunk *mb_chunk);                        /* ref :2070-2075 */
int32_t duckdb_mb_is_null_data_chunk(duckdb_mb_data_chunk *mb_chunk);                   /* ref :2077-2079 */
void *duckdb_mb_vector_get_data(duckdb_vector vector);                                  /* ref :2085-2087 */
uint64_t *duckdb_mb_vector_get_validity(duckdb_vector vector);                          /* ref :2089-2091 */
duckdb_vector duckdb_mb_list_vector_get_child(duckdb_vector vector);                    /* ref :2093-2095 */
duckdb_state duckdb_mb_list_vector_set_size(duckdb_vector vector, idx_t size);          /* ref :2097-2099 */
duckdb_state duckdb_mb_list_vector_reserve(duckdb_vector vector, idx_t capacity);       /* ref :2101-2103 */
int32_t duckdb_mb_append_data_chunk(duckdb_mb_appender *mb_append, duckdb_mb_data_chunk *mb_chunk); /* ref :2109-2132 */

/* Bound-plan cache of a prepared SELECT: out2[0] = times the statement was
 * bound, out2[1] = executions that reused the bound plan with only the
 * parameter constants overwritten.  Returns 1 on success. */
int32_t duckdb_mbx_statement_plan_stats(duckdb_mb_statement *statement, int64_t *out2);

/* Partial aggregate export for multi-GPU combine: the i-th cell of the last
 * materialized result as raw little-endian bytes (HUGEINT: 16 bytes). */
int32_t duckdb_mbx_result_raw(duckdb_mb_result *result, int32_t col, int32_t row, void *out, int32_t out_len);

/* Every cell of a result as text in one call — the strings and NULL flags of
 * duckdb_mb_result_is_null/_value (ref src/duckdb_native.c:216-238) for the
 * per-cell loop of Connection::query (src/duckdb_native.mbt:477-497).
 * Layout: i64 nrows, i64 ncols, u8 null[nrows*ncols] row-major, zero pad to 8,
 * i64 offsets[nrows*ncols+1], chars.  malloc'd: free with duckdb_mbx_free. */
char *duckdb_mbx_result_text(duckdb_mb_result *result, int64_t *len);

/* Counters of the in-library multi-device path (Config::set "gpu_devices",
 * the key rides ref src/duckdb_native.c:714-747): out6 = {shards, peer-access
 * links enabled at connect, shard dispatches, peer DMA copies, peer DMA bytes,
 * sharded aggregates finished on the host}; outd2 = {last dispatch wall us,
 * last host merge us}.  Either pointer may be NULL.  Returns 6 (0: no handle). */
int32_t duckdb_mbx_shard_stats(duckdb_mb_connection *connection, int64_t *out6, double *outd2);

/* One-pass selection (select_rounds) outcomes over the connection and its
 * shards: out3 = {launches, aborts (a persistent workgroup was never scheduled
 * within 100 ms, so the query reran in the two-pass form), launch failures (the
 * two-pass form ran instead)}.  Returns 3 (0: no handle). */
int32_t duckdb_mbx_engine_stats(duckdb_mb_connection *connection, int64_t *out3);

/* The last sharded dispatch, per shard i: out[4 i .. 4 i + 3] = {device,
 * wake_us, launch_us, done_us}, us since the dispatch began (the worker took
 * the job; its plan and launches were queued; its result reached the host:
 * kernel + D2H + synchronisation).  At most cap shards are written; returns
 * the dispatch's shard count (0: none yet). */
int32_t duckdb_mbx_shard_timings(duckdb_mb_connection *connection, double *out, int32_t cap);

/* Shard i's partial aggregate relation of the last sharded aggregate, as it
 * left its device before the merge (groups, then COUNT / SUM / MIN / MAX
 * partials; AVG as SUM then COUNT).  Read it with the duckdb_mb_result_*
 * accessors and free it with duckdb_mb_result_destroy; NULL if none. */
duckdb_mb_result *duckdb_mbx_shard_partial(duckdb_mb_connection *connection, int32_t shard);

/* mbx_combine=rccl (the default; Config::set key, ref src/duckdb_native.c:714-747): a
 * sharded global aggregate over distinct devices is combined by RCCL on the
 * shard devices (ncclInt64 reduce to device 0 for COUNT-only rows; all-gather of int128
 * lanes + a carry-correct combine on device 0 otherwise).  out2 = {RCCL
 * combines, requests that fell back to the host merge}; out_us1 = the last
 * combine's collective + D2H wall us.  Returns 2 (0: no handle). */
int32_t duckdb_mbx_rccl_stats(duckdb_mb_connection *connection, int64_t *out2, double *out_us1);
/* Why the last RCCL request fell back ("" if it ran); free with duckdb_mbx_free. */
char *duckdb_mbx_rccl_note(duckdb_mb_connection *connection);
/* Up to cap of {RCCL combines, host-merge fallbacks (a combine RCCL should
 * have run: communicators unavailable, a collective failed or timed out),
 * combines through the test loopback, combines that raised a shard's device
 * error, collectives aborted after MBX_RCCL_TIMEOUT_MS (default 20 s; the host
 * merge answers), combines of GROUP BY relations (one integer key: dense key
 * slots all-gathered), requests RCCL never covers (floating-point partials,
 * non-integer or several keys, same-device shards), ncclReduce combines,
 * ncclAllGather combines}; returns the count written. */
int32_t duckdb_mbx_rccl_stats_ex(duckdb_mb_connection *connection, int64_t *out, int32_t cap);
/* 1: RCCL combine, 0: host merge, from the next statement on; 2: the RCCL
 * combine with its collectives replaced by device copies (tests only: refused
 * without MBX_EXPERIMENTS=1), so it runs over same-device shards.  Returns 1
 * (0: refused). */
int32_t duckdb_mbx_set_combine(duckdb_mb_connection *connection, int32_t mode);
/* The RCCL calls the combine makes, checked on hardware: a fresh
 * ncclCommInitAll over `device` alone (one rank), then the multi-rank check the
 * combine is gated on (one grouped ncclReduce and one ncclAllGather of 97 int64
 * lanes, verified on every rank).  Returns 1 and the wall microseconds in
 * *us_out (may be NULL); 0 with the reason in duckdb_mb_last_error(). */
int32_t duckdb_mbx_rccl_selftest(int32_t device, double *us_out);
/* The same over n distinct devices (n ranks): a JSON object {"ok", "error",
 * "devices", "init_us", "check_us", "total_us", "ranks": [{"device", "count",
 * "user_rank", "cu_device"}]} where count / user_rank / cu_device are what
 * ncclCommCount / ncclCommUserRank / ncclCommCuDevice report (-1 if librccl
 * lacks the query).  Free with duckdb_mbx_free. */
char *duckdb_mbx_rccl_selftest_ex(const int32_t *devices, int32_t n);
/* The connection's RCCL combine as a JSON object: the combine mode, the
 * communicators' state ("none" / "pending" / "ready" / "failed" / "loopback"),
 * whether their open started at connect, its ncclCommInitAll seconds and
 * check microseconds, how long the first combine waited for it, every rank's
 * ncclCommCount / ncclCommUserRank / ncclCommCuDevice, the counters of
 * duckdb_mbx_rccl_stats_ex and the collective the last combine ran.  Free
 * with duckdb_mbx_free. */
char *duckdb_mbx_rccl_info(duckdb_mb_connection *connection);
/* The RCCL combine's lane arithmetic on the host (tests): gathered holds
 * nranks x (3 ncols + 1) int64 lanes ({lo, hi, non-NULL} per column, then the
 * rank's error word); kinds[j] = 0 sum / 1 min / 2 max; out = 3 ncols lanes.
 * Returns 1 (0: bad arguments). */
int32_t duckdb_mbx_combine_lanes(const int64_t *gathered, int32_t nranks, int32_t ncols, const int8_t *kinds,
                                 int64_t *out);

#ifdef __cplusplus
}
#endif

#endif /* DUCKDB_MB_AMD_H */
