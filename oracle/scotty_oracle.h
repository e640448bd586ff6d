/*
 * scotty_oracle.h -- C API of the CPU ORACLE (test infrastructure only).
 *
 * This library is a single-threaded restatement of the reference Java
 * SlicingWindowOperator (julianev/scotty-window-processor v0.4).  It exists
 * to CHECK the MI355X product path (libscotty_mi355x.so); only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product never links, calls or falls back to it.
 *
 * Every function below names the reference method it restates in oracle.cpp.
 */
#ifndef SCOTTY_ORACLE_H
#define SCOTTY_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* window kinds (core/windowType) */
#define ORC_WIN_TUMBLING 0
#define ORC_WIN_SLIDING 1
#define ORC_WIN_SESSION 2
#define ORC_WIN_FIXED_BAND 3
#define ORC_WIN_TEST_SCRIPTED 100 /* SliceManagerTest.TestWindow (T/SliceManagerTest.java:297-368) */
#define ORC_WIN_TEST_NULLCTX 101  /* SliceFactoryTest.TestWindow, createContext()==null (:492-509) */

#define ORC_MEASURE_TIME 0
#define ORC_MEASURE_COUNT 1

/* aggregate kinds (value semantics of the demo / benchmark functions) */
#define ORC_AGG_SUM_I32 0  /* (a,b)->a+b on Integer (int32 wrap) */
#define ORC_AGG_COUNT 1    /* demo Count: lift=1, combine=+ (int32 wrap) */
#define ORC_AGG_MIN_I32 2  /* Math.min */
#define ORC_AGG_MAX_I32 3  /* Math.max */
#define ORC_AGG_SUM_I64 4
#define ORC_AGG_MIN_I64 5
#define ORC_AGG_MAX_I64 6
#define ORC_AGG_SUM_F64 7
#define ORC_AGG_MIN_F64 8
#define ORC_AGG_MAX_F64 9
#define ORC_AGG_FIRST 10   /* the arrival index of the first partial's tuple (include/scotty_mi355x.h SCOTTY_AGG_FIRST) */
#define ORC_AGG_SUB_I32 100 /* (a,b)->a-b (TumblingWindowOperatorTest.java:212) */
/* OR-able flag: function implements InvertibleAggregateFunction */
#define ORC_AGG_INVERTIBLE 0x10000

/* state factories */
#define ORC_STATE_MEMORY 0 /* MemoryStateFactory */
#define ORC_STATE_MOCK 1   /* T/StateFactoryMock.java: ValueState never empty */

/* error codes (Java exception that the reference would throw) */
#define ORC_OK 0
#define ORC_ERR_INDEX -1    /* IndexOutOfBoundsException */
#define ORC_ERR_NPE -2      /* NullPointerException */
#define ORC_ERR_NOELEM -3   /* NoSuchElementException */
#define ORC_ERR_ARITH -4    /* ArithmeticException (/ by zero) */
#define ORC_ERR_ARG -5      /* bad argument to the oracle API itself */
#define ORC_ERR_HANG -6     /* the reference would loop forever (StreamSlicer, see oracle.cpp) */

typedef struct orc_op orc_op;

typedef struct {
  int64_t t_start, t_end, t_first, t_last, c_start, c_last;
  int32_t type_fixed; /* 1 = Slice.Fixed, 0 = Slice.Flexible */
  int32_t flex_count;
  int32_t is_lazy;
  int32_t n_records;
} orc_slice_info;

orc_op* orc_create(int state_mode);
void orc_destroy(orc_op*);
const char* orc_last_error(orc_op*);
/* order in which a Set<WindowModifications> is iterated: 0 insertion, 1 reverse, 2 seeded shuffle */
void orc_set_mod_order(orc_op*, int mode, uint64_t seed);

int orc_add_window(orc_op*, int kind, int measure, int64_t a, int64_t b);
int orc_add_aggregation(orc_op*, int kind);
int orc_set_max_lateness(orc_op*, int64_t);

/* SlicingWindowOperator.processElement(element, ts); value_i used by integer aggs, value_f by f64 */
int orc_process_element(orc_op*, int64_t value_i, double value_f, int64_t ts);
/* convenience: n elements in arrival order (value_f may be NULL) */
int orc_process_elements(orc_op*, const int64_t* ts, const int64_t* value_i, const double* value_f,
                         size_t n, size_t* n_failed);
/* SlicingWindowOperator.processWatermark(wm); results kept until the next call */
int orc_process_watermark(orc_op*, int64_t wm);
int64_t orc_num_windows(orc_op*);
int orc_window(orc_op*, int64_t i, int64_t* start, int64_t* end, int32_t* measure, int32_t* has_value,
               int32_t* n_values);
/* value j of window i (j indexes getAggValues(), i.e. non-empty functions only).
 * is_null set when the lowered value is Java null (StateFactoryMock). */
int orc_window_value(orc_op*, int64_t i, int32_t j, int64_t* vi, double* vf, int32_t* is_null);

/* --- component-level hooks used by SliceManagerTest / SliceFactoryTest / LazyAggregateStoreTest --- */
int orc_store_size(orc_op*);
int orc_slice(orc_op*, int idx, orc_slice_info* out);
int orc_slice_records(orc_op*, int idx, int64_t* ts_out, int cap);
int orc_slice_value(orc_op*, int idx, int32_t j, int64_t* vi, double* vf, int32_t* is_null);
int orc_slice_num_values(orc_op*, int idx);
/* aggregationStore.appendSlice(sliceFactory.createSlice(start, end, type)) */
int orc_store_append_new_slice(orc_op*, int64_t start, int64_t end, int type_fixed, int flex_count);
/* sliceFactory.createSlice(...) instanceof LazySlice */
int orc_factory_would_be_lazy(orc_op*);
/* sliceManager.processElement(element, ts) (no StreamSlicer) */
int orc_manager_process_element(orc_op*, int64_t value_i, int64_t ts);
int orc_store_find_slice_index_by_ts(orc_op*, int64_t ts);
int orc_store_insert_value_to_slice(orc_op*, int idx, int64_t value_i, int64_t ts);
int orc_store_insert_value_to_current(orc_op*, int64_t value_i, int64_t ts);
/* WindowManager flags: bit0 hasContextAware, bit1 isSessionWindowCase, bit2 hasCountMeasure,
 * bit3 hasFixedWindows, bit4 hasTimeMeasure */
int orc_manager_flags(orc_op*);
int64_t orc_max_lateness(orc_op*);
int64_t orc_current_count(orc_op*);

/* --- keyed connector (KeyedScottyWindowOperator.java:41-86) on T threads: CPU baseline of the keyed config --- */
typedef struct orc_keyed orc_keyed;
orc_keyed* orc_keyed_create(int threads);
void orc_keyed_destroy(orc_keyed*);
int orc_keyed_add_window(orc_keyed*, int kind, int measure, int64_t a, int64_t b);
int orc_keyed_add_aggregation(orc_keyed*, int kind);
int orc_keyed_set_max_lateness(orc_keyed*, int64_t);
int64_t orc_keyed_num_keys(orc_keyed*);
/* partition t = rows [off[t], off[t+1]); returns forwarded (hasValue) windows or a negative error */
int64_t orc_keyed_process(orc_keyed*, const int64_t* off, const uint32_t* keys, const int64_t* ts,
                          const int64_t* value_i, int64_t watermark);

#ifdef __cplusplus
}
#endif
#endif
