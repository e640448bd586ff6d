// scotty_oracle.cpp -- CPU ORACLE for the Scotty general-stream-slicing path.
//
// TEST INFRASTRUCTURE ONLY.  A single-threaded, line-by-line restatement of the
// reference Java operator (julianev/scotty-window-processor v0.4, read-only at
// /root/reference).  It is the checker for the MI355X product library and is
// never linked into it.  Java semantics kept on purpose: int/long wrap-around,
// truncating %, the Long.MAX_VALUE first-edge overflow, TreeSet-by-ts record
// de-duplication, ArrayList index exceptions, tLast-based window containment.
// Java exceptions are modelled as C++ exceptions thrown at the same point, so
// the state the reference would leave behind is reproduced as well.
//
// Citation prefixes (relative to /root/reference):
//   S/  slicing/src/main/java/de/tub/dima/scotty/slicing/
//   C/  core/src/main/java/de/tub/dima/scotty/core/
//   ST/ state/src/main/java/de/tub/dima/scotty/state/
#include "scotty_oracle.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

using i64 = int64_t;
constexpr i64 JMAX = INT64_MAX;
constexpr i64 JMIN = INT64_MIN;

struct JavaException {
  int code;
  std::string msg;
};
[[noreturn]] void throw_index(const std::string& m) { throw JavaException{ORC_ERR_INDEX, "IndexOutOfBoundsException: " + m}; }
[[noreturn]] void throw_npe(const std::string& m) { throw JavaException{ORC_ERR_NPE, "NullPointerException: " + m}; }
[[noreturn]] void throw_noelem(const std::string& m) { throw JavaException{ORC_ERR_NOELEM, "NoSuchElementException: " + m}; }
[[noreturn]] void throw_cce(const std::string& m) { throw JavaException{ORC_ERR_NPE, "ClassCastException: " + m}; }

inline i64 jadd(i64 a, i64 b) { return (i64)((uint64_t)a + (uint64_t)b); }
inline i64 jsub(i64 a, i64 b) { return (i64)((uint64_t)a - (uint64_t)b); }
inline int32_t iadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
inline int32_t isub(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }
inline i64 jmod(i64 a, i64 b) {  // Java long %, truncating
  if (b == 0) throw JavaException{ORC_ERR_ARITH, "ArithmeticException: / by zero"};
  if (b == -1) return 0;
  return a % b;
}
// Math.min / Math.max on double (NaN propagates, -0.0 < +0.0)
inline double jmin_d(double a, double b) {
  if (a != a) return a;
  if (a == 0.0 && b == 0.0 && std::signbit(b)) return b;
  return a <= b ? a : b;
}
inline double jmax_d(double a, double b) {
  if (a != a) return a;
  if (a == 0.0 && b == 0.0 && std::signbit(a)) return b;
  return a >= b ? a : b;
}

// ---------------------------------------------------------------- elements
struct Elem {
  i64 i = 0;
  double f = 0.0;
  i64 seq = 0;  // arrival index (processElement calls before this one): the value ORC_AGG_FIRST lifts
};
// S/slice/StreamRecord.java:3-33 -- compareTo by ts only (:25-27)
struct Record {
  i64 ts;
  Elem e;
};
struct RecordLess {
  bool operator()(const Record& a, const Record& b) const { return a.ts < b.ts; }
};
using RecordSet = std::set<Record, RecordLess>;  // ST/memory/MemorySetState.java:9 TreeSet

// ---------------------------------------------------------------- functions
// C/windowFunction/AggregateFunction.java (lift :17, combine :34, liftAndCombine :44-47, lower :56),
// InvertibleAggregateFunction.java (invert :10, liftAndInvert :12-15).  Concrete semantics follow the
// demo / benchmark functions: SumAggregation (B/flinkBenchmark/aggregations/SumAggregation.java:16-18),
// Count (D/*/windowFunctions/Count.java), Min/MaxWindowFunction (Math.min / Math.max).
struct Partial {
  bool null_ = true;
  i64 i = 0;
  double f = 0.0;
};
struct AggFn {
  int kind;
  bool invertible;
  bool is_f64() const { return kind == ORC_AGG_SUM_F64 || kind == ORC_AGG_MIN_F64 || kind == ORC_AGG_MAX_F64; }
  Partial lift(const Elem& e) const {
    Partial p;
    p.null_ = false;
    switch (kind) {
      case ORC_AGG_COUNT: p.i = 1; break;
      case ORC_AGG_SUM_I32: case ORC_AGG_MIN_I32: case ORC_AGG_MAX_I32: case ORC_AGG_SUB_I32:
        p.i = (int32_t)e.i; break;
      case ORC_AGG_SUM_I64: case ORC_AGG_MIN_I64: case ORC_AGG_MAX_I64: p.i = e.i; break;
      case ORC_AGG_FIRST: p.i = e.seq; break;
      default: p.f = e.f; break;
    }
    return p;
  }
  Partial combine(const Partial& a, const Partial& b) const {
    if (a.null_ || b.null_) throw_npe("combine(null)");  // Integer unboxing of null
    Partial r;
    r.null_ = false;
    switch (kind) {
      case ORC_AGG_SUM_I32: case ORC_AGG_COUNT: r.i = iadd((int32_t)a.i, (int32_t)b.i); break;
      case ORC_AGG_SUB_I32: r.i = isub((int32_t)a.i, (int32_t)b.i); break;
      case ORC_AGG_MIN_I32: case ORC_AGG_MIN_I64: r.i = std::min(a.i, b.i); break;
      case ORC_AGG_MAX_I32: case ORC_AGG_MAX_I64: r.i = std::max(a.i, b.i); break;
      case ORC_AGG_SUM_I64: r.i = jadd(a.i, b.i); break;
      case ORC_AGG_SUM_F64: r.f = a.f + b.f; break;
      case ORC_AGG_MIN_F64: r.f = jmin_d(a.f, b.f); break;
      case ORC_AGG_MAX_F64: r.f = jmax_d(a.f, b.f); break;
      // a combine that keeps partialAggregate1's fields (B/flinkBenchmark/aggregations/SumAggregation.java:16-18,
      // D/flink-demo/.../SumWindowFunction.java:16-17): the partial's identifying tuple stays the first one
      case ORC_AGG_FIRST: r.i = a.i; break;
    }
    return r;
  }
  Partial liftAndCombine(const Partial& p, const Elem& e) const { return combine(p, lift(e)); }
  Partial invert(const Partial& a, const Partial& b) const {
    if (a.null_ || b.null_) throw_npe("invert(null)");
    Partial r;
    r.null_ = false;
    switch (kind) {
      case ORC_AGG_SUM_I32: case ORC_AGG_COUNT: r.i = isub((int32_t)a.i, (int32_t)b.i); break;
      case ORC_AGG_SUM_I64: r.i = jsub(a.i, b.i); break;
      case ORC_AGG_SUM_F64: r.f = a.f - b.f; break;
      default: r = a; break;  // not reachable: only sums are declared invertible
    }
    return r;
  }
};

// ---------------------------------------------------------------- state
// ValueState: ST/memory/MemoryValueState.java (null <=> empty, :27-29; clean sets null :17-19)
//             T/StateFactoryMock.java:9-36 (isEmpty() always false, clean() no-op)
struct ValueState {
  bool mock = false;
  Partial v;
  bool isEmpty() const { return mock ? false : v.null_; }
  void clean() {
    if (!mock) v = Partial();
  }
};

// S/state/AggregateValueState.java
struct AggregateValueState {
  ValueState ps;
  const AggFn* fn;
  const RecordSet* records;  // null for eager slices / windows
  // :23-31
  void addElement(const Elem& e) {
    if (ps.isEmpty() || ps.v.null_) ps.v = fn->lift(e);
    else ps.v = fn->liftAndCombine(ps.v, e);
  }
  // :33-41
  void removeElement(const Record* rec) {
    if (fn->invertible) {
      if (rec == nullptr) throw_npe("streamRecord.record");
      ps.v = fn->invert(ps.v, fn->lift(rec->e));
    } else {
      recompute();
    }
  }
  // :43-49
  void recompute() {
    clean();
    if (records)
      for (const Record& r : *records) addElement(r.e);
  }
  void clean() { ps.clean(); }
  // :55-69 (clone of the partial is the identity for value-typed partials)
  void merge(const AggregateValueState& o) {
    if (ps.isEmpty() && !o.ps.isEmpty()) {
      ps.v = o.ps.v;
    } else if (!o.ps.isEmpty()) {
      ps.v = fn->combine(ps.v, o.ps.v);
    }
  }
  bool hasValue() const { return !ps.isEmpty(); }
};

// S/state/AggregateState.java
struct AggregateState {
  std::vector<AggregateValueState> vs;
  AggregateState() = default;
  AggregateState(bool mock, const std::vector<std::unique_ptr<AggFn>>& fns, const RecordSet* records) {
    for (auto& f : fns) {
      AggregateValueState s;
      s.ps.mock = mock;
      s.fn = f.get();
      s.records = records;
      vs.push_back(s);
    }
  }
  void addElement(const Elem& e) {  // :25-29
    for (auto& s : vs) s.addElement(e);
  }
  void removeElement(const Record* r) {  // :31-35
    for (auto& s : vs) s.removeElement(r);
  }
  void merge(const AggregateState& o) {  // :44-50
    if (o.vs.size() <= vs.size())
      for (size_t i = 0; i < o.vs.size(); i++) vs[i].merge(o.vs[i]);
  }
  bool hasValues() const {  // :56-63
    for (auto& s : vs)
      if (s.hasValue()) return true;
    return false;
  }
};

// ---------------------------------------------------------------- slices
// S/slice/Slice.java -- Type: Fixed (:86-92) or Flexible(counter) (:94-121), movable <=> counter==1.
struct SliceType {
  bool fixed = false;
  int counter = 1;
  bool isMovable() const { return !fixed && counter == 1; }
  static SliceType Fixed() { SliceType t; t.fixed = true; t.counter = 0; return t; }
  static SliceType Flexible(int c = 1) { SliceType t; t.fixed = false; t.counter = c; return t; }
};

// S/slice/AbstractSlice.java + EagerSlice.java + LazySlice.java
struct Slice {
  i64 tStart, tEnd;
  SliceType type;
  i64 tLast, tFirst = JMAX;
  i64 cStart, cLast;
  bool lazy;
  std::unique_ptr<RecordSet> records;  // LazySlice only
  AggregateState state;
  Slice(i64 s, i64 e, i64 cs, i64 cl, SliceType t, bool lz, bool mock, const std::vector<std::unique_ptr<AggFn>>& fns)
      : tStart(s), tEnd(e), type(t), tLast(s), cStart(cs), cLast(cl), lazy(lz) {  // AbstractSlice :16-23
    if (lazy) records.reset(new RecordSet());
    state = AggregateState(mock, fns, records.get());
  }
  void absAdd(i64 ts) {  // AbstractSlice.addElement :27-31
    tLast = std::max(tLast, ts);
    tFirst = std::min(tFirst, ts);
    cLast = jadd(cLast, 1);
  }
  void addElement(const Elem& e, i64 ts) {
    absAdd(ts);
    state.addElement(e);                   // EagerSlice :23-26 / LazySlice :23-27
    if (lazy) records->insert(Record{ts, e});
  }
  void prependElement(const Record* r) {  // LazySlice :29-33
    if (!lazy) throw_cce("EagerSlice cannot be cast to LazySlice");
    if (!r) throw_npe("prependElement(null)");
    absAdd(r->ts);
    records->insert(*r);
    state.addElement(r->e);
  }
  // LazySlice.dropLastElement :35-44
  bool dropLastElement(Record* out) {
    if (!lazy) throw_cce("EagerSlice cannot be cast to LazySlice");
    bool have = !records->empty();
    Record rec{};
    if (have) {
      auto it = std::prev(records->end());
      rec = *it;
      records->erase(it);
    }
    cLast = jsub(cLast, 1);
    if (!records->empty()) tLast = std::prev(records->end())->ts;
    state.removeElement(have ? &rec : nullptr);
    if (out) *out = rec;
    return have;
  }
  // LazySlice.dropFirstElement :46-53
  bool dropFirstElement(Record* out) {
    if (!lazy) throw_cce("EagerSlice cannot be cast to LazySlice");
    bool have = !records->empty();
    Record rec{};
    if (have) {
      rec = *records->begin();
      records->erase(records->begin());
    }
    if (records->empty()) throw_noelem("TreeSet.first()");
    i64 first = records->begin()->ts;
    cLast = jsub(cLast, 1);
    tFirst = first;
    state.removeElement(have ? &rec : nullptr);
    if (out) *out = rec;
    return have;
  }
  void merge(const Slice& o) {  // AbstractSlice.merge :34-39
    tLast = std::max(tLast, o.tLast);
    tFirst = std::min(tFirst, o.tFirst);
    tEnd = std::max(tEnd, o.tEnd);
    state.merge(o.state);
  }
};

// ---------------------------------------------------------------- windows
struct Mod {  // C/windowType/windowContext/{Add,Delete,Shift}Modification.java
  int kind;   // 0 shift, 1 delete, 2 add
  i64 pre, post;
};
struct ActiveWindow {
  i64 start, end;
};

struct WindowCollector;

// C/windowType/windowContext/WindowContext.java
struct WindowContext {
  std::vector<ActiveWindow> active;
  std::vector<Mod>* mods = nullptr;
  std::vector<Mod> stale;  // sink for modifications recorded outside updateContext
  int measure = ORC_MEASURE_TIME;
  virtual ~WindowContext() = default;
  bool hasActiveWindows() const { return active.empty(); }  // :15-17 (sic: returns isEmpty())
  std::vector<Mod>& M() { return mods ? *mods : stale; }
  size_t addNewWindow(size_t i, i64 start, i64 end) {  // :19-25
    if (i > active.size()) throw_index("activeWindows.add(" + std::to_string(i) + ")");
    active.insert(active.begin() + i, ActiveWindow{start, end});
    M().push_back(Mod{2, 0, start});
    M().push_back(Mod{2, 0, end});
    return i;
  }
  ActiveWindow& getWindow(long i) {
    if (i < 0 || (size_t)i >= active.size()) throw_index("activeWindows.get(" + std::to_string(i) + ")");
    return active[i];
  }
  int numberOfActiveWindows() const { return (int)active.size(); }
  void mergeWithPre(int idx) {  // :39-46
    ActiveWindow w = getWindow(idx);
    ActiveWindow& pre = getWindow(idx - 1);
    shiftEnd(pre, w.end);
    removeWindow(idx);
  }
  void removeWindow(int idx) {  // :48-52
    ActiveWindow& w = getWindow(idx);
    M().push_back(Mod{1, w.start, 0});
    M().push_back(Mod{1, w.end, 0});
    active.erase(active.begin() + idx);
  }
  void shiftStart(ActiveWindow& w, i64 pos) {  // :55-58
    M().push_back(Mod{0, w.start, pos});
    w.start = pos;
  }
  void shiftEnd(ActiveWindow& w, i64 pos) { w.end = pos; }  // :60-63 (records no modification)
  void updateContext(const Elem& e, i64 pos, std::vector<Mod>* m) {  // :68-71
    mods = m;
    update(e, pos);
    mods = nullptr;  // later removeWindow() calls write to a stale set (never read)
  }
  virtual void update(const Elem& e, i64 pos) = 0;
  virtual i64 assignNextWindowStart(i64 pos) = 0;
  virtual void triggerWindows(WindowCollector& c, i64 lastWm, i64 wm) = 0;
};

struct WindowCollector {
  // S/WindowManager.java:204-227 AggregationWindowCollector
  struct Win {
    i64 start, end;
    int measure;
    AggregateState st;
  };
  std::vector<Win> wins;
  bool mock;
  const std::vector<std::unique_ptr<AggFn>>* fns;
  void trigger(i64 s, i64 e, int measure) {  // :209-212 -> AggregateWindowState ctor
    wins.push_back(Win{s, e, measure, AggregateState(mock, *fns, nullptr)});
  }
};

// C/windowType/SessionWindow.java:40-116 (SessionContext)
struct SessionContext : WindowContext {
  i64 gap;
  void update(const Elem&, i64 position) override {  // :42-87
    if (hasActiveWindows()) {
      addNewWindow(0, position, position);
      return;
    }
    int sessionIndex = getSession(position);
    if (sessionIndex == -1) {
      addNewWindow(0, position, position);
    } else {
      ActiveWindow& s = getWindow(sessionIndex);
      if (jsub(s.start, gap) > position) {
        addNewWindow(sessionIndex, position, position);
      } else if (s.start > position && jsub(s.start, gap) < position) {
        shiftStart(s, position);
        if (sessionIndex > 0) {
          ActiveWindow& pre = getWindow(sessionIndex - 1);
          if (jadd(pre.end, gap) >= getWindow(sessionIndex).start) {
            mergeWithPre(sessionIndex);
            return;
          }
        }
      } else if (s.end < position && jadd(s.end, gap) >= position) {
        shiftEnd(s, position);
        if (sessionIndex < numberOfActiveWindows() - 1) {
          ActiveWindow& next = getWindow(sessionIndex + 1);
          if (jadd(getWindow(sessionIndex).end, gap) >= next.start) {
            mergeWithPre(sessionIndex + 1);
            return;
          }
        }
      } else if (jadd(s.end, gap) < position) {
        addNewWindow(sessionIndex + 1, position, position);
      }
    }
  }
  int getSession(i64 position) {  // :89-101
    int i = 0;
    for (; i < numberOfActiveWindows(); i++) {
      ActiveWindow& s = getWindow(i);
      if (jsub(s.start, gap) <= position && jadd(s.end, gap) >= position) return i;
      else if (jsub(s.start, gap) > position) return i - 1;
    }
    return i - 1;
  }
  i64 assignNextWindowStart(i64 p) override { return jadd(p, gap); }  // :104-106
  void triggerWindows(WindowCollector& c, i64, i64 wm) override {  // :108-119
    ActiveWindow s = getWindow(0);
    while (jadd(s.end, gap) < wm) {
      c.trigger(s.start, jadd(s.end, gap), measure);
      removeWindow(0);
      if (hasActiveWindows()) return;
      s = getWindow(0);
    }
  }
};

// T/SliceManagerTest.java:310-362 (scripted context-aware test window)
struct ScriptedContext : WindowContext {
  void update(const Elem&, i64 position) override {
    int index = getWindowIndex(position);
    if (index == -1) {
      addNewWindow(0, jsub(position, jmod(position, 10)), jsub(jadd(position, 10), jmod(position, 10)));
      return;
    } else if (jmod(position, 5) != 0 && position > getWindow(index).end) {
      addNewWindow(index + 1, jsub(position, jmod(position, 10)), jsub(jadd(position, 10), jmod(position, 10)));
      return;
    }
    if (position == 5) {
      shiftStart(getWindow(index + 1), position);
    } else if (position == 15) {
      shiftStart(getWindow(index), position);
    } else if (position == 25) {
      addNewWindow(index, position, jsub(jadd(position, 10), jmod(position, 10)));
    } else if (position == 35) {
      mergeWithPre(index);
    }
  }
  int getWindowIndex(i64 position) {
    int i = 0;
    for (; i < numberOfActiveWindows(); i++) {
      ActiveWindow& s = getWindow(i);
      if (s.start <= position && s.end > position) return i;
    }
    return i - 1;
  }
  i64 assignNextWindowStart(i64 p) override { return jsub(jadd(p, 10), jmod(p, 10)); }
  void triggerWindows(WindowCollector& c, i64, i64 wm) override {
    ActiveWindow w = getWindow(0);
    while (w.end <= wm) {
      c.trigger(w.start, w.end, measure);
      removeWindow(0);
      if (hasActiveWindows()) return;
      w = getWindow(0);
    }
  }
};

// C/windowType/{Tumbling,Sliding,FixedBand}Window.java (ContextFreeWindow)
struct CFWindow {
  int kind, measure;
  i64 a, b;  // tumbling: size | sliding: size, slide | fixed band: start, size
  i64 assignNextWindowStart(i64 t) const {
    switch (kind) {
      case ORC_WIN_TUMBLING: return jsub(jadd(t, a), jmod(t, a));              // TumblingWindow :29-31
      case ORC_WIN_SLIDING: return jsub(jadd(t, b), jmod(t, b));               // SlidingWindow :41-43
      default:                                                                 // FixedBandWindow :37-48
        if (t == JMAX || t < a) return a;
        if (t >= a && t < jadd(a, b)) return jadd(a, b);
        return JMAX;
    }
  }
  void triggerWindows(WindowCollector& c, i64 lastWm, i64 wm) const {
    if (kind == ORC_WIN_TUMBLING) {  // TumblingWindow :34-39
      i64 size = a;
      i64 lastStart = jsub(lastWm, jmod(jadd(lastWm, size), size));
      for (i64 ws = lastStart; jadd(ws, size) <= wm; ws = jadd(ws, size)) c.trigger(ws, jadd(ws, size), measure);
    } else if (kind == ORC_WIN_SLIDING) {  // SlidingWindow :45-57
      i64 size = a, slide = b;
      i64 lastStart = jsub(wm, jmod(jadd(wm, slide), slide));
      for (i64 ws = lastStart; jadd(ws, size) > lastWm; ws = jsub(ws, slide))
        if (ws >= 0 && jadd(ws, size) <= jadd(wm, 1)) c.trigger(ws, jadd(ws, size), measure);
    } else {  // FixedBandWindow :51-57
      i64 ws = a;
      if (lastWm <= jadd(ws, b) && jadd(ws, b) <= wm) c.trigger(ws, jadd(ws, b), measure);
    }
  }
  i64 clearDelay() const { return kind == ORC_WIN_FIXED_BAND ? b : a; }
};

// ---------------------------------------------------------------- operator
struct Op {
  bool mock;
  int mod_order = 0;
  std::mt19937_64 rng{1};
  std::string err;
  // WindowManager fields (S/WindowManager.java:18-33)
  bool hasContextAwareWindows = false, hasFixedWindows = false, hasCountMeasure = false;
  bool hasTimeMeasure = false, isSessionWindowCase = false;
  i64 maxLateness = 1000, maxFixedWindowSize = 0, lastWatermark = -1, currentCount = 0, lastCount = 0;
  std::vector<CFWindow> contextFreeWindows;
  std::vector<std::unique_ptr<WindowContext>> contextAwareWindows;  // entries may be null (NULLCTX)
  std::vector<std::unique_ptr<AggFn>> windowFunctions;
  // LazyAggregateStore (S/aggregationstore/LazyAggregateStore.java)
  std::vector<std::unique_ptr<Slice>> slices;
  // StreamSlicer fields (S/StreamSlicer.java:10-14)
  i64 maxEventTime = JMIN, min_next_edge_ts = JMIN, min_next_edge_count = JMIN;
  // last watermark result
  std::vector<WindowCollector::Win> result;

  // ---- AggregationStore
  Slice& getSlice(long i) {
    if (i < 0 || (size_t)i >= slices.size()) throw_index("slices.get(" + std::to_string(i) + ")");
    return *slices[i];
  }
  Slice& getCurrentSlice() { return getSlice((long)slices.size() - 1); }
  int findSliceIndexByTimestamp(i64 ts) {  // :29-37
    for (int i = (int)slices.size() - 1; i >= 0; i--)
      if (slices[i]->tStart <= ts) return i;
    return -1;
  }
  int findSliceIndexByCount(i64 c) {  // :41-49
    for (int i = (int)slices.size() - 1; i >= 0; i--)
      if (slices[i]->cStart <= c) return i;
    return -1;
  }
  int findSliceByEnd(i64 e) {  // :127-135
    for (int i = (int)slices.size() - 1; i >= 0; i--)
      if (slices[i]->tEnd == e) return i;
    return -1;
  }
  void mergeSlice(int idx) {  // :119-124
    Slice& a = getSlice(idx);
    Slice& b = getSlice(idx + 1);
    a.merge(b);
    slices.erase(slices.begin() + idx + 1);
  }
  void removeSlices(i64 t) {  // :138-146
    int idx = findSliceIndexByTimestamp(t);
    if (idx <= 0) return;
    slices.erase(slices.begin(), slices.begin() + idx);
  }
  void addSlice(size_t idx, std::unique_ptr<Slice> s) {
    if (idx > slices.size()) throw_index("slices.add(" + std::to_string(idx) + ")");
    slices.insert(slices.begin() + idx, std::move(s));
  }

  // ---- SliceFactory (S/slice/SliceFactory.java:17-22)
  bool factoryLazy() const {
    return !(!hasCountMeasure && ((!hasContextAwareWindows || isSessionWindowCase) && maxLateness > 0));
  }
  std::unique_ptr<Slice> createSlice(i64 s, i64 e, i64 cs, i64 cl, SliceType t) {
    return std::unique_ptr<Slice>(new Slice(s, e, cs, cl, t, factoryLazy(), mock, windowFunctions));
  }

  // ---- WindowManager.addWindowAssigner (S/WindowManager.java:121-147)
  void addWindowAssigner(int kind, int measure, i64 a, i64 b) {
    if (kind == ORC_WIN_TUMBLING || kind == ORC_WIN_SLIDING || kind == ORC_WIN_FIXED_BAND) {
      CFWindow w{kind, measure, a, b};
      contextFreeWindows.push_back(w);
      maxFixedWindowSize = std::max(maxFixedWindowSize, w.clearDelay());
      hasFixedWindows = true;
    } else {  // ForwardContextAware
      bool isSession = kind == ORC_WIN_SESSION;
      if (isSession && (!hasContextAwareWindows || isSessionWindowCase)) isSessionWindowCase = true;
      else isSessionWindowCase = false;
      hasContextAwareWindows = true;
      std::unique_ptr<WindowContext> ctx;
      if (kind == ORC_WIN_SESSION) {
        auto* s = new SessionContext();
        s->gap = a;
        ctx.reset(s);
      } else if (kind == ORC_WIN_TEST_SCRIPTED) {
        ctx.reset(new ScriptedContext());
      }
      if (ctx) ctx->measure = measure;
      contextAwareWindows.push_back(std::move(ctx));
    }
    if (measure == ORC_MEASURE_COUNT) hasCountMeasure = true;
    else hasTimeMeasure = true;
  }

  // ---- SliceManager (S/SliceManager.java)
  void appendSlice(i64 startTs, SliceType type) {  // :27-38
    if (!slices.empty()) {
      Slice& cur = getCurrentSlice();
      cur.tEnd = startTs;
      cur.type = type;
    }
    slices.push_back(createSlice(startTs, JMAX, currentCount, currentCount, SliceType::Flexible()));
  }
  WindowContext& ctxAt(size_t i) {
    if (!contextAwareWindows[i]) throw_npe("createContext() returned null");
    return *contextAwareWindows[i];
  }
  void orderMods(std::vector<Mod>& m) {
    if (mod_order == 1) std::reverse(m.begin(), m.end());
    else if (mod_order == 2) std::shuffle(m.begin(), m.end(), rng);
  }
  void managerProcessElement(const Elem& e, i64 ts) {  // :47-87
    if (slices.empty()) appendSlice(0, SliceType::Flexible());
    Slice& cur = getCurrentSlice();
    if (ts >= cur.tLast) {
      cur.addElement(e, ts);  // insertValueToCurrentSlice
      std::vector<Mod> discard;  // new HashSet per tuple; modifications dropped (:59-62)
      for (size_t i = 0; i < contextAwareWindows.size(); i++) ctxAt(i).updateContext(e, ts, &discard);
    } else {
      for (size_t i = 0; i < contextAwareWindows.size(); i++) {
        std::vector<Mod> mods;
        ctxAt(i).updateContext(e, ts, &mods);
        orderMods(mods);
        checkSliceEdges(mods);
      }
      int idx = findSliceIndexByTimestamp(ts);
      getSlice(idx).addElement(e, ts);
      if (hasCountMeasure) {  // :77-85 shift count in slices
        for (; idx <= (int)slices.size() - 2; idx++) {
          Slice& ls = getSlice(idx);
          Record r;
          bool have = ls.dropLastElement(&r);
          Slice& nx = getSlice(idx + 1);
          nx.prependElement(have ? &r : nullptr);
        }
      }
    }
  }
  void checkSliceEdges(const std::vector<Mod>& mods) {  // :89-166
    for (const Mod& mod : mods) {
      if (mod.kind == 0) {  // ShiftModification
        i64 pre = mod.pre, post = mod.post;
        int sliceIndex = findSliceByEnd(pre);
        if (sliceIndex == -1) continue;
        Slice* cur = &getSlice(sliceIndex);
        SliceType st = cur->type;
        if (st.isMovable()) {
          Slice* next = &getSlice(sliceIndex + 1);
          cur->tEnd = post;
          next->tStart = post;
          if (post < pre) {
            if (cur->lazy) {
              while (cur->tFirst < cur->tLast && cur->tLast >= post) {
                Record r;
                bool have = cur->dropLastElement(&r);
                next->prependElement(have ? &r : nullptr);
              }
            }
          } else {
            if (cur->lazy) {
              while (next->tFirst < next->tLast && next->tFirst < post) {
                Record r;
                bool have = next->dropFirstElement(&r);
                cur->prependElement(have ? &r : nullptr);
              }
            }
          }
        } else {
          if (!cur->type.fixed) cur->type.counter--;
          splitSlice(sliceIndex, post);
        }
      }
      if (mod.kind == 1) {  // DeleteModification
        int sliceIndex = findSliceByEnd(mod.pre);
        if (sliceIndex >= 0) {
          Slice* cur = &getSlice(sliceIndex);
          if (cur->type.isMovable()) {
            Slice* next = &getSlice(sliceIndex + 1);
            if (next->lazy) {
              while (next->cLast > 0) {
                Record r;
                bool have = next->dropLastElement(&r);
                cur->prependElement(have ? &r : nullptr);
              }
            }
            mergeSlice(sliceIndex);
          } else {
            if (!cur->type.fixed) cur->type.counter--;
          }
        }
      }
      if (mod.kind == 2) {  // AddModification
        i64 edge = mod.post;
        int sliceIndex = findSliceIndexByTimestamp(edge);
        Slice& s = getSlice(sliceIndex);
        if (s.tStart != edge && s.tEnd != edge) splitSlice(sliceIndex, edge);
      }
    }
  }
  void splitSlice(int sliceIndex, i64 timestamp) {  // :168-192
    Slice* a = &getSlice(sliceIndex);
    Slice* b = nullptr;
    if (timestamp < a->tEnd) {
      auto nb = createSlice(timestamp, a->tEnd, a->cStart, a->cLast, a->type);
      a->tEnd = timestamp;
      a->type = SliceType::Flexible();
      b = nb.get();
      addSlice(sliceIndex + 1, std::move(nb));
      a = &getSlice(sliceIndex);
    } else if (sliceIndex + 1 < (int)slices.size()) {
      a = &getSlice(sliceIndex + 1);
      auto nb = createSlice(timestamp, a->tEnd, a->cStart, a->cLast, a->type);
      a->tEnd = timestamp;
      a->type = SliceType::Flexible();
      b = nb.get();
      addSlice(sliceIndex + 2, std::move(nb));
      a = &getSlice(sliceIndex + 1);
    } else {
      return;
    }
    if (a->lazy) {
      while (a->tLast >= timestamp) {
        Record r;
        bool have = a->dropLastElement(&r);
        b->prependElement(have ? &r : nullptr);
      }
    }
  }

  // ---- StreamSlicer (S/StreamSlicer.java:36-141)
  i64 calculateNextFixedEdgeCount() {  // :88-101
    i64 cur = min_next_edge_count == JMIN ? 0 : min_next_edge_count;
    i64 t_c = std::max(currentCount, cur);
    i64 edge = JMAX;
    for (auto& w : contextFreeWindows)
      if (w.measure == ORC_MEASURE_COUNT) edge = std::min(w.assignNextWindowStart(t_c), edge);
    return edge;
  }
  i64 calculateNextFixedEdge(i64 te) {  // :103-116
    i64 cur = min_next_edge_ts == JMIN ? JMAX : min_next_edge_ts;
    i64 t_c = std::max(jsub(te, maxLateness), cur);
    i64 edge = JMAX;
    for (auto& w : contextFreeWindows)
      if (w.measure == ORC_MEASURE_TIME) edge = std::min(w.assignNextWindowStart(t_c), edge);
    return edge;
  }
  int calculateNextFlexEdge(i64 te) {  // :118-130
    i64 t_c = std::max(maxEventTime, min_next_edge_ts);
    int flex = 0;
    for (size_t i = 0; i < contextAwareWindows.size(); i++)
      if (te >= ctxAt(i).assignNextWindowStart(t_c)) flex++;
    return flex;
  }
  void determineSlices(i64 te) {  // :36-86
    if (hasCountMeasure) {
      if (min_next_edge_count == JMIN || currentCount == min_next_edge_count) {
        if (maxEventTime == JMIN) maxEventTime = te;
        appendSlice(maxEventTime, SliceType::Fixed());
        min_next_edge_count = calculateNextFixedEdgeCount();
      }
    }
    if (hasTimeMeasure) {
      bool inOrder = te >= maxEventTime;
      if (inOrder) {
        if (hasFixedWindows && min_next_edge_ts == JMIN) min_next_edge_ts = calculateNextFixedEdge(te);
        int flex = 0;
        if (hasContextAwareWindows) flex = calculateNextFlexEdge(te);
        while (hasFixedWindows && te > min_next_edge_ts) {
          if (min_next_edge_ts >= 0) appendSlice(min_next_edge_ts, SliceType::Fixed());
          min_next_edge_ts = calculateNextFixedEdge(te);
          // If the minimum assignNextWindowStart is exactly Long.MIN_VALUE (a power-of-two tumbling size or
          // sliding slide wraps Long.MAX_VALUE + 1 on the first call), calculateNextFixedEdge treats the edge
          // as "unset" again and the reference spins in this loop forever.  Report instead of hanging.
          if (min_next_edge_ts == JMIN)
            throw JavaException{ORC_ERR_HANG, "reference StreamSlicer loops forever: calculateNextFixedEdge "
                                              "returned Long.MIN_VALUE (power-of-two window size/slide)"};
        }
        if (min_next_edge_ts == te) {
          if (flex > 0) appendSlice(te, SliceType::Fixed());
          else appendSlice(min_next_edge_ts, SliceType::Fixed());
          min_next_edge_ts = calculateNextFixedEdge(te);
        } else if (flex > 0) {
          appendSlice(te, SliceType::Flexible(flex));
        }
      }
    }
    currentCount = jadd(currentCount, 1);  // WindowManager.incrementCount :196-198
    maxEventTime = std::max(te, maxEventTime);
  }

  // ---- SlicingWindowOperator.processElement (S/SlicingWindowOperator.java:41-44)
  i64 arrivals = 0;  // processElement calls so far (the arrival index ORC_AGG_FIRST lifts)
  void processElement(const Elem& e, i64 ts) {
    Elem x = e;
    x.seq = arrivals++;
    determineSlices(ts);
    managerProcessElement(x, ts);
  }

  // ---- LazyAggregateStore.aggregate (:83-111) + AggregateWindowState.containsSlice (:25-31)
  void aggregate(std::vector<WindowCollector::Win>& wins, i64 minTs, i64 maxTs, i64 minCount, i64 maxCount) {
    int startIndex = std::max(findSliceIndexByTimestamp(minTs), 0);
    startIndex = std::min(startIndex, findSliceIndexByCount(minCount));
    int endIndex = std::min((int)slices.size() - 1, findSliceIndexByTimestamp(maxTs));
    endIndex = std::max(endIndex, findSliceIndexByCount(maxCount));
    for (int i = startIndex; i <= endIndex; i++) {
      Slice& s = getSlice(i);
      for (auto& w : wins) {
        bool contains = w.measure == ORC_MEASURE_TIME ? (w.start <= s.tStart && w.end > s.tLast)
                                                      : (w.start <= s.cStart && w.end >= s.cLast);
        if (contains) w.st.merge(s.state);
      }
    }
  }

  // ---- WindowManager.processWatermark (S/WindowManager.java:41-118)
  void processWatermark(i64 wm) {
    result.clear();
    if (lastWatermark == -1) lastWatermark = std::max((i64)0, jsub(wm, maxLateness));
    if (slices.empty()) {
      lastWatermark = wm;
      return;
    }
    i64 oldest = getSlice(0).tStart;
    if (lastWatermark < oldest) lastWatermark = oldest;
    WindowCollector col;
    col.mock = mock;
    col.fns = &windowFunctions;
    for (auto& w : contextFreeWindows) {  // assignContextFreeWindows :104-118
      if (w.measure == ORC_MEASURE_TIME) {
        w.triggerWindows(col, lastWatermark, wm);
      } else {
        int idx = findSliceIndexByTimestamp(wm);
        Slice* s = &getSlice(idx);
        if (s->tLast >= wm && idx > 0) s = &getSlice(idx - 1);
        i64 cend = s->cLast;
        w.triggerWindows(col, lastCount, jadd(cend, 1));
      }
    }
    for (size_t i = 0; i < contextAwareWindows.size(); i++)  // assignContextAwareWindows :98-102
      ctxAt(i).triggerWindows(col, lastWatermark, wm);
    i64 minTs = JMAX, maxTs = 0, minCount = currentCount, maxCount = 0;
    for (auto& w : col.wins) {
      if (w.measure == ORC_MEASURE_TIME) {
        minTs = std::min(w.start, minTs);
        maxTs = std::max(w.end, maxTs);
      } else {
        minCount = std::min(w.start, minCount);
        maxCount = std::max(w.end, maxCount);
      }
    }
    if (!col.wins.empty()) aggregate(col.wins, minTs, maxTs, minCount, maxCount);
    lastWatermark = wm;
    lastCount = currentCount;
    clearAfterWatermark(jsub(wm, maxLateness));
    result = std::move(col.wins);
  }
  void clearAfterWatermark(i64 cw) {  // :82-95
    i64 first = cw;
    for (size_t i = 0; i < contextAwareWindows.size(); i++)
      for (auto& a : ctxAt(i).active) first = std::min(first, a.start);
    i64 maxDelay = jsub(cw, maxFixedWindowSize);
    removeSlices(std::min(maxDelay, first));
  }
};

}  // namespace

struct orc_op {
  Op op;
};

template <class F>
static int guarded(orc_op* o, F&& f) {
  try {
    f();
    return ORC_OK;
  } catch (JavaException& e) {
    o->op.err = e.msg;
    return e.code;
  }
}

static void fill_partial(const Partial& p, const AggFn* fn, int64_t* vi, double* vf, int32_t* is_null) {
  if (is_null) *is_null = p.null_ ? 1 : 0;
  if (vi) *vi = p.i;
  if (vf) *vf = fn->is_f64() ? p.f : (double)p.i;
}

extern "C" {

orc_op* orc_create(int state_mode) {
  orc_op* o = new orc_op();
  o->op.mock = state_mode == ORC_STATE_MOCK;
  return o;
}
void orc_destroy(orc_op* o) { delete o; }
const char* orc_last_error(orc_op* o) { return o->op.err.c_str(); }
void orc_set_mod_order(orc_op* o, int mode, uint64_t seed) {
  o->op.mod_order = mode;
  o->op.rng.seed(seed);
}

int orc_add_window(orc_op* o, int kind, int measure, int64_t a, int64_t b) {
  if ((kind == ORC_WIN_TUMBLING && a <= 0) || (kind == ORC_WIN_SLIDING && (a <= 0 || b <= 0)) ||
      (kind == ORC_WIN_SESSION && a < 0)) {
    o->op.err = "window size/slide/gap must be positive";
    return ORC_ERR_ARG;
  }
  if (kind != ORC_WIN_TUMBLING && kind != ORC_WIN_SLIDING && kind != ORC_WIN_SESSION && kind != ORC_WIN_FIXED_BAND &&
      kind != ORC_WIN_TEST_SCRIPTED && kind != ORC_WIN_TEST_NULLCTX) {
    o->op.err = "unknown window kind";
    return ORC_ERR_ARG;
  }
  return guarded(o, [&] { o->op.addWindowAssigner(kind, measure, a, b); });
}
int orc_add_aggregation(orc_op* o, int kind) {
  int base = kind & 0xFFFF;
  bool inv = (kind & ORC_AGG_INVERTIBLE) != 0;
  bool ok = (base >= ORC_AGG_SUM_I32 && base <= ORC_AGG_MAX_F64) || base == ORC_AGG_SUB_I32 || base == ORC_AGG_FIRST;
  if (!ok || (inv && !(base == ORC_AGG_SUM_I32 || base == ORC_AGG_COUNT || base == ORC_AGG_SUM_I64 ||
                       base == ORC_AGG_SUM_F64))) {
    o->op.err = "unknown / non-invertible aggregation kind";
    return ORC_ERR_ARG;
  }
  o->op.windowFunctions.emplace_back(new AggFn{base, inv});
  return (int)o->op.windowFunctions.size() - 1;
}
int orc_set_max_lateness(orc_op* o, int64_t l) {
  o->op.maxLateness = l;
  return ORC_OK;
}
int orc_process_element(orc_op* o, int64_t vi, double vf, int64_t ts) {
  Elem e{vi, vf};
  return guarded(o, [&] { o->op.processElement(e, ts); });
}
int orc_process_elements(orc_op* o, const int64_t* ts, const int64_t* vi, const double* vf, size_t n,
                         size_t* n_failed) {
  size_t failed = 0;
  int first = ORC_OK;
  for (size_t k = 0; k < n; k++) {
    Elem e{vi ? vi[k] : 0, vf ? vf[k] : (vi ? (double)vi[k] : 0.0)};
    int rc = guarded(o, [&] { o->op.processElement(e, ts[k]); });
    if (rc != ORC_OK) {
      failed++;
      if (first == ORC_OK) first = rc;
    }
  }
  if (n_failed) *n_failed = failed;
  return first;
}
int orc_process_watermark(orc_op* o, int64_t wm) {
  return guarded(o, [&] { o->op.processWatermark(wm); });
}
int64_t orc_num_windows(orc_op* o) { return (int64_t)o->op.result.size(); }
int orc_window(orc_op* o, int64_t i, int64_t* start, int64_t* end, int32_t* measure, int32_t* has_value,
               int32_t* n_values) {
  if (i < 0 || (size_t)i >= o->op.result.size()) return ORC_ERR_INDEX;
  auto& w = o->op.result[i];
  if (start) *start = w.start;
  if (end) *end = w.end;
  if (measure) *measure = w.measure;
  if (has_value) *has_value = w.st.hasValues() ? 1 : 0;
  int nv = 0;
  for (auto& s : w.st.vs)
    if (s.hasValue()) nv++;
  if (n_values) *n_values = nv;
  return ORC_OK;
}
int orc_window_value(orc_op* o, int64_t i, int32_t j, int64_t* vi, double* vf, int32_t* is_null) {
  if (i < 0 || (size_t)i >= o->op.result.size()) return ORC_ERR_INDEX;
  auto& w = o->op.result[i];
  int k = 0;
  for (auto& s : w.st.vs) {  // AggregateState.getValues :65-72 (skips empty)
    if (!s.hasValue()) continue;
    if (k == j) {
      fill_partial(s.ps.v, s.fn, vi, vf, is_null);
      return ORC_OK;
    }
    k++;
  }
  return ORC_ERR_INDEX;
}

int orc_store_size(orc_op* o) { return (int)o->op.slices.size(); }
int orc_slice(orc_op* o, int idx, orc_slice_info* out) {
  if (idx < 0 || (size_t)idx >= o->op.slices.size()) return ORC_ERR_INDEX;
  Slice& s = *o->op.slices[idx];
  out->t_start = s.tStart;
  out->t_end = s.tEnd;
  out->t_first = s.tFirst;
  out->t_last = s.tLast;
  out->c_start = s.cStart;
  out->c_last = s.cLast;
  out->type_fixed = s.type.fixed ? 1 : 0;
  out->flex_count = s.type.counter;
  out->is_lazy = s.lazy ? 1 : 0;
  out->n_records = s.lazy ? (int32_t)s.records->size() : 0;
  return ORC_OK;
}
int orc_slice_records(orc_op* o, int idx, int64_t* ts_out, int cap) {
  if (idx < 0 || (size_t)idx >= o->op.slices.size()) return ORC_ERR_INDEX;
  Slice& s = *o->op.slices[idx];
  if (!s.lazy) return 0;
  int k = 0;
  for (auto& r : *s.records) {
    if (k < cap) ts_out[k] = r.ts;
    k++;
  }
  return k;
}
int orc_slice_num_values(orc_op* o, int idx) {
  if (idx < 0 || (size_t)idx >= o->op.slices.size()) return ORC_ERR_INDEX;
  int nv = 0;
  for (auto& s : o->op.slices[idx]->state.vs)
    if (s.hasValue()) nv++;
  return nv;
}
int orc_slice_value(orc_op* o, int idx, int32_t j, int64_t* vi, double* vf, int32_t* is_null) {
  if (idx < 0 || (size_t)idx >= o->op.slices.size()) return ORC_ERR_INDEX;
  int k = 0;
  for (auto& s : o->op.slices[idx]->state.vs) {
    if (!s.hasValue()) continue;
    if (k == j) {
      fill_partial(s.ps.v, s.fn, vi, vf, is_null);
      return ORC_OK;
    }
    k++;
  }
  return ORC_ERR_INDEX;
}
int orc_store_append_new_slice(orc_op* o, int64_t start, int64_t end, int type_fixed, int flex_count) {
  SliceType t = type_fixed ? SliceType::Fixed() : SliceType::Flexible(flex_count);
  o->op.slices.push_back(o->op.createSlice(start, end, o->op.currentCount, o->op.currentCount, t));
  return ORC_OK;
}
int orc_factory_would_be_lazy(orc_op* o) { return o->op.factoryLazy() ? 1 : 0; }
int orc_manager_process_element(orc_op* o, int64_t vi, int64_t ts) {
  Elem e{vi, (double)vi};
  return guarded(o, [&] { o->op.managerProcessElement(e, ts); });
}
int orc_store_find_slice_index_by_ts(orc_op* o, int64_t ts) { return o->op.findSliceIndexByTimestamp(ts); }
int orc_store_insert_value_to_slice(orc_op* o, int idx, int64_t vi, int64_t ts) {
  Elem e{vi, (double)vi};
  return guarded(o, [&] { o->op.getSlice(idx).addElement(e, ts); });
}
int orc_store_insert_value_to_current(orc_op* o, int64_t vi, int64_t ts) {
  Elem e{vi, (double)vi};
  return guarded(o, [&] { o->op.getCurrentSlice().addElement(e, ts); });
}
int orc_manager_flags(orc_op* o) {
  Op& p = o->op;
  return (p.hasContextAwareWindows ? 1 : 0) | (p.isSessionWindowCase ? 2 : 0) | (p.hasCountMeasure ? 4 : 0) |
         (p.hasFixedWindows ? 8 : 0) | (p.hasTimeMeasure ? 16 : 0);
}
int64_t orc_max_lateness(orc_op* o) { return o->op.maxLateness; }
int64_t orc_current_count(orc_op* o) { return o->op.currentCount; }

// ---- keyed connector (flink-connector/.../KeyedScottyWindowOperator.java:41-86): one operator per key, created on
//      first sight (:56-62); a watermark is processed by every key's operator (:72-86), which forwards only hasValue()
//      windows (:80).  The CPU baseline runs T partitions of the key space on T threads (what an upstream keyBy with
//      parallelism T delivers): partition t owns rows [off[t], off[t+1]) of the arrays.
struct orc_keyed {
  struct WinSpec {
    int kind, measure;
    int64_t a, b;
  };
  std::vector<WinSpec> wins;
  std::vector<int> aggs;
  int64_t lateness = 1000;
  int threads = 1;
  std::vector<std::unordered_map<uint32_t, orc_op*>> maps;
};

orc_keyed* orc_keyed_create(int threads) {
  orc_keyed* k = new orc_keyed();
  k->threads = threads < 1 ? 1 : threads;
  k->maps.resize(k->threads);
  return k;
}
void orc_keyed_destroy(orc_keyed* k) {
  if (!k) return;
  for (auto& m : k->maps)
    for (auto& kv : m) delete kv.second;
  delete k;
}
int orc_keyed_add_window(orc_keyed* k, int kind, int measure, int64_t a, int64_t b) {
  k->wins.push_back({kind, measure, a, b});
  return ORC_OK;
}
int orc_keyed_add_aggregation(orc_keyed* k, int kind) {
  k->aggs.push_back(kind);
  return ORC_OK;
}
int orc_keyed_set_max_lateness(orc_keyed* k, int64_t l) {
  k->lateness = l;
  return ORC_OK;
}
int64_t orc_keyed_num_keys(orc_keyed* k) {
  int64_t n = 0;
  for (auto& m : k->maps) n += (int64_t)m.size();
  return n;
}
// processElement of every row (arrival order within each partition), then processWatermark(wm) of every key's
// operator.  Returns the number of forwarded (hasValue) windows, or a negative Java error code.
int64_t orc_keyed_process(orc_keyed* k, const int64_t* off, const uint32_t* keys, const int64_t* ts,
                          const int64_t* vi, int64_t wm) {
  std::vector<int64_t> emitted(k->threads, 0);
  std::vector<int> errs(k->threads, ORC_OK);
  auto work = [&](int t) {
    auto& mp = k->maps[t];
    for (int64_t r = off[t]; r < off[t + 1]; r++) {
      auto it = mp.find(keys[r]);
      orc_op* o;
      if (it == mp.end()) {  // initWindowOperator() (:57-60)
        o = orc_create(ORC_STATE_MEMORY);
        for (auto& w : k->wins) orc_add_window(o, w.kind, w.measure, w.a, w.b);
        for (int a : k->aggs) orc_add_aggregation(o, a);
        orc_set_max_lateness(o, k->lateness);
        mp.emplace(keys[r], o);
      } else {
        o = it->second;
      }
      Elem e{vi[r], (double)vi[r]};
      const int rc = guarded(o, [&] { o->op.processElement(e, ts[r]); });
      if (rc != ORC_OK && errs[t] == ORC_OK) errs[t] = rc;
    }
    for (auto& kv : mp) {
      orc_op* o = kv.second;
      const int rc = guarded(o, [&] { o->op.processWatermark(wm); });
      if (rc != ORC_OK) {
        if (errs[t] == ORC_OK) errs[t] = rc;
        continue;
      }
      for (auto& w : o->op.result)
        if (w.st.hasValues()) emitted[t]++;
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < k->threads; t++) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
  int64_t tot = 0;
  for (int t = 0; t < k->threads; t++) {
    if (errs[t] != ORC_OK) return errs[t];
    tot += emitted[t];
  }
  return tot;
}

}  // extern "C"
