package de.tub.dima.scotty.slicing;

import de.tub.dima.scotty.core.AggregateWindow;
import de.tub.dima.scotty.core.WindowOperator;
import de.tub.dima.scotty.core.windowFunction.AggregateFunction;
import de.tub.dima.scotty.core.windowType.FixedBandWindow;
import de.tub.dima.scotty.core.windowType.SessionWindow;
import de.tub.dima.scotty.core.windowType.SlidingWindow;
import de.tub.dima.scotty.core.windowType.TumblingWindow;
import de.tub.dima.scotty.core.windowType.Window;
import de.tub.dima.scotty.core.windowType.WindowMeasure;
import de.tub.dima.scotty.state.StateFactory;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.ArrayList;
import java.util.HashMap;
import java.util.List;

/**
 * Drop-in for the reference's {@code de.tub.dima.scotty.slicing.SlicingWindowOperator}
 * (slicing/src/main/java/de/tub/dima/scotty/slicing/SlicingWindowOperator.java:20-70), backed by
 * {@code libscotty_mi355x.so} (C-ABI: include/scotty_mi355x.h) through {@link NativeApi}: JNI by default (any JDK from
 * 8, the reference's target), or the Java 22 FFM API from the optional {@code java/ffm} source set.  Java 8 source.
 * Put this class ahead of the reference's slicing jar on the classpath; the connectors'
 * {@code new SlicingWindowOperator<>(stateFactory)} then binds here, unchanged.
 *
 * <p>Two modes, chosen at construction:
 * <ul>
 *   <li>a stand-alone operator (GlobalScottyWindowOperator, direct users): one native operator; processElement
 *       appends to an off-heap buffer (no native call) which goes to the GPU as one micro-batch
 *       (scotty_process_elements) before the next processWatermark or configuration call;</li>
 *   <li>a per-key operator of a keyed connector (recognised by {@link KeyedEngine#sharedForCaller}, or opted in with
 *       {@link #perKey} / {@link #keyedScope()} / {@code -Dscotty.keyed.engine=on}): the instance is one key of its
 *       thread's shared keyed native operator ({@link KeyedEngine}): one push and one native watermark per watermark
 *       round for all keys.</li>
 * </ul>
 * Window results come back as SoA columns, in the reference's emission order, and are rebuilt into
 * {@link NativeAggregateWindow}s whose values are the objects the functions' lower() returns
 * ({@link NativeFunctions.Binding#rebuild}).  Only functions with a GPU binding run ({@link NativeFunctions#bind});
 * anything else is rejected with UnsupportedOperationException at addAggregation -- there is no CPU fallback.
 */
public class SlicingWindowOperator<InputType> implements WindowOperator<InputType> {

    // SCOTTY_WIN_* / SCOTTY_FLAG_KEYED / error codes of include/scotty_mi355x.h
    static final int WIN_TUMBLING = 0, WIN_SLIDING = 1, WIN_SESSION = 2, WIN_FIXED_BAND = 3;
    static final int FLAG_KEYED = 1;
    static final int ERR_INDEX = -5;

    private final transient NativeApi api = NativeApi.get();
    private final int valueType, width;
    private final NativeValues.Extractor<InputType> extractor;  // null: the functions' bindings read the value
    private final List<NativeFunctions.Binding> bindings = new ArrayList<NativeFunctions.Binding>();
    private final List<long[]> windows = new ArrayList<long[]>();      // {kind, measure, a, b} in registration order
    private long maxLateness = 1000;                              // S/WindowManager.java:24
    private boolean latenessSet = false;
    private final boolean keyed;
    // stand-alone mode: the native operator and the off-heap micro-batch (created in the constructor on the task
    // that runs the operator: connectors build operators in open(), not by deserialization)
    private transient long op;
    private transient ByteBuffer tsBuf, valBuf;
    private long buffered = 0;
    // keyed mode: the shared engine and this instance's key
    private transient KeyedEngine engine;
    private int id = -1;
    // stand-alone mode, functions whose result keeps the window's first partial's fields (NativeFunctions.Binding
    // #keepsFirst): the hidden SCOTTY_AGG_FIRST column gives each window the arrival index of that tuple; the tuples
    // since the last watermark and the first tuples of the retained slices (scotty_first_indices) are kept to rebuild
    private final List<Integer> colOf = new ArrayList<Integer>();  // native result column of each binding
    private int firstCol = -1;
    private long arrivals = 0, recentBase = 0;
    private transient ArrayList<Object> recent = new ArrayList<Object>();
    private transient HashMap<Long, Object> retained = new HashMap<Long, Object>();

    /** S/SlicingWindowOperator.java:30-37: the state factory is not used (slices live in HBM). */
    public SlicingWindowOperator(StateFactory stateFactory) {
        this(stateFactory, NativeValues.VALUE_I32, null);
    }

    /**
     * valueType: NativeValues.VALUE_I32 / VALUE_I64 / VALUE_F64; extractor: the numeric value of a tuple (null: the
     * registered functions' bindings read it).  Per-key or stand-alone as {@link KeyedEngine#sharedForCaller} decides.
     */
    public SlicingWindowOperator(StateFactory stateFactory, int valueType, NativeValues.Extractor<InputType> extractor) {
        this(valueType, extractor, KeyedEngine.sharedForCaller());
    }

    private SlicingWindowOperator(int valueType, NativeValues.Extractor<InputType> extractor, boolean keyed) {
        this.valueType = valueType;
        this.width = valueType == NativeValues.VALUE_I32 ? 4 : 8;
        this.extractor = extractor;
        this.keyed = keyed;
        if (!keyed) {
            this.op = api.create(0, valueType, 0);
            allocate(1 << 16);
        }
    }

    /**
     * Explicit opt-in: the operator of ONE key of a keyed wrapper -- every instance created this way on a thread (with
     * equal configuration) shares that thread's keyed native operator ({@link KeyedEngine}).  For new keyed code; the
     * reference's connectors are recognised without it.
     */
    public static <T> SlicingWindowOperator<T> perKey(StateFactory stateFactory, int valueType,
                                                      NativeValues.Extractor<T> extractor) {
        return new SlicingWindowOperator<T>(valueType, extractor, true);
    }

    /**
     * Explicit opt-in for an unchanged keyed wrapper the shim does not recognise by name: every SlicingWindowOperator
     * constructed on this thread until the returned scope is closed is a per-key instance.
     * {@code try (SlicingWindowOperator.KeyedScope s = SlicingWindowOperator.keyedScope()) { wrapper.open(); }}
     */
    public static KeyedScope keyedScope() {
        KeyedEngine.SCOPE.get()[0]++;
        return new KeyedScope();
    }

    /** See {@link #keyedScope()}. */
    public static final class KeyedScope implements AutoCloseable {
        private boolean open = true;

        private KeyedScope() {
        }

        @Override
        public void close() {
            if (open) {
                open = false;
                KeyedEngine.SCOPE.get()[0]--;
            }
        }
    }

    @Override
    public void processElement(InputType element, long ts) {
        Number v = value(element);
        if (keyed) {
            bindEngine();
            engine.add(id, ts, v);
            return;
        }
        if (firstCol >= 0) recent.add(element);
        arrivals++;
        if (buffered == tsBuf.capacity() / 8) allocate(2 * buffered);
        tsBuf.putLong((int) (8 * buffered), ts);
        if (valueType == NativeValues.VALUE_I32) valBuf.putInt((int) (4 * buffered), v.intValue());
        else if (valueType == NativeValues.VALUE_I64) valBuf.putLong((int) (8 * buffered), v.longValue());
        else valBuf.putDouble((int) (8 * buffered), v.doubleValue());
        buffered++;
    }

    /** S/SlicingWindowOperator.java:46-49 (WindowManager.processWatermark, S/WindowManager.java:38-61). */
    @Override
    public List<AggregateWindow> processWatermark(long watermarkTs) {
        if (keyed) {
            bindEngine();
            List<KeyedEngine.Row> rows = engine.watermark(id, watermarkTs);
            List<AggregateWindow> out = new ArrayList<AggregateWindow>(rows.size());
            for (KeyedEngine.Row r : rows) out.add(window(r.start, r.end, r.measure, r.has, r.words, null));
            return out;
        }
        flush();
        NativeApi.Windows w = new NativeApi.Windows();
        check(api.processWatermark(op, watermarkTs, w));
        List<AggregateWindow> out = new ArrayList<AggregateWindow>(w.n);
        for (int i = 0; i < w.n; i++) {
            long[] words = new long[bindings.size()];
            for (int k = 0; k < words.length; k++) words[k] = w.values[colOf.get(k)][i];
            Object first = firstCol >= 0 && w.has[i] != 0 ? payload(w.values[firstCol][i]) : null;
            out.add(window(w.start[i], w.end[i], w.measure[i], w.has[i] != 0, words, first));
        }
        if (firstCol >= 0) retainFirsts();
        return out;
    }

    private AggregateWindow window(long start, long end, int measure, boolean has, long[] words, Object first) {
        List<Object> agg = new ArrayList<Object>(words.length);
        if (has)
            for (int k = 0; k < words.length; k++) agg.add(bindings.get(k).rebuild(words[k], first));
        return new NativeAggregateWindow(measure == 0 ? WindowMeasure.Time : WindowMeasure.Count, start, end, has, agg);
    }

    /** The tuple with arrival index {@code index}: this interval's, or a retained slice's first tuple. */
    private Object payload(long index) {
        Object t = index >= recentBase ? recent.get((int) (index - recentBase)) : retained.get(index);
        if (t == null)
            throw new IllegalStateException("first partial's tuple " + index + " is neither in this interval nor a "
                    + "retained slice's first tuple");
        return t;
    }

    /** After a watermark: keep only the tuples a later window can still return as its first partial's. */
    private void retainFirsts() {
        long[] keep = api.firstIndices(op);
        if (keep == null) throw new UnsupportedOperationException(api.lastError(op));
        HashMap<Long, Object> next = new HashMap<Long, Object>(2 * keep.length + 1);
        for (long x : keep) next.put(x, payload(x));
        retained = next;
        recent.clear();
        recentBase = arrivals;
    }

    /** WindowManager.addWindowAssigner (S/WindowManager.java:121-147). */
    @Override
    public void addWindowAssigner(Window window) {
        long[] w = describe(window);
        windows.add(w);
        if (keyed) {
            configuredAfterUse();
            return;
        }
        flush();
        check(api.addWindow(op, (int) w[0], (int) w[1], w[2], w[3]));
    }

    private static long[] describe(Window window) {
        int m = window.getWindowMeasure() == WindowMeasure.Time ? 0 : 1;
        if (window instanceof TumblingWindow)
            return new long[]{WIN_TUMBLING, m, ((TumblingWindow) window).getSize(), 0L};
        if (window instanceof SlidingWindow) {
            SlidingWindow s = (SlidingWindow) window;
            return new long[]{WIN_SLIDING, m, s.getSize(), s.getSlide()};
        }
        if (window instanceof SessionWindow)
            return new long[]{WIN_SESSION, m, ((SessionWindow) window).getGap(), 0L};
        if (window instanceof FixedBandWindow) {
            FixedBandWindow f = (FixedBandWindow) window;
            return new long[]{WIN_FIXED_BAND, m, f.getStart(), f.getSize()};
        }
        throw new UnsupportedOperationException("window type without a GPU kind: " + window);
    }

    /** WindowManager.addAggregation (S/WindowManager.java:196-198). */
    @Override
    public <OutputType> void addAggregation(AggregateFunction<InputType, ?, OutputType> windowFunction) {
        NativeFunctions.Binding b = NativeFunctions.bind(windowFunction, valueType);
        if (keyed && b.needsFirst())
            throw new UnsupportedOperationException(windowFunction.getClass().getName() + " keeps the window's first "
                    + "partial's fields, which the keyed engine does not track (SCOTTY_AGG_FIRST runs on stand-alone "
                    + "operators)");
        bindings.add(b);
        if (keyed) {
            colOf.add(bindings.size() - 1);
            configuredAfterUse();
            return;
        }
        // SCOTTY_AGG_FIRST runs on the grid path: every window a context-free time window (the connectors register
        // the windows before the function, F/GlobalScottyWindowOperator.java:40-47)
        boolean grid = true;
        for (long[] w : windows) grid &= w[0] != WIN_SESSION && w[1] == 0;
        if (b.needsFirst() && !grid)
            throw new UnsupportedOperationException(windowFunction.getClass().getName() + " keeps the window's first "
                    + "partial's fields: SCOTTY_AGG_FIRST needs context-free time windows only (no session or count "
                    + "windows)");
        flush();
        colOf.add(check(api.addAggregation(op, b.kind)));
        if (b.keepsFirst() && grid && firstCol < 0)
            firstCol = check(api.addAggregation(op, NativeValues.AGG_FIRST));
    }

    /** S/SlicingWindowOperator.java:57-63. */
    public <Agg, OutputType> void addWindowFunction(AggregateFunction<InputType, Agg, OutputType> windowFunction) {
        addAggregation(windowFunction);
    }

    @Override
    public void setMaxLateness(long maxLateness) {
        this.maxLateness = maxLateness;
        this.latenessSet = true;
        if (keyed) {
            configuredAfterUse();
            return;
        }
        flush();
        check(api.setMaxLateness(op, maxLateness));
    }

    /** Frees the native operator (stand-alone mode; a keyed engine lives as long as its thread). */
    public void close() {
        if (!keyed && op != 0) {
            api.destroy(op);
            op = 0;
        }
    }

    // ---- value of a tuple: the explicit extractor, else the first value-reading binding (all must agree)
    private Number value(InputType element) {
        if (extractor != null) {
            for (NativeFunctions.Binding b : bindings) b.value(element);  // exemplars / key checks
            return valueType == NativeValues.VALUE_F64 ? (Number) extractor.doubleValue(element)
                    : (Number) extractor.value(element);
        }
        Number v = null;
        for (NativeFunctions.Binding b : bindings) {
            Number x = b.value(element);
            if ((b.kind & 0xFFFF) == NativeValues.AGG_COUNT) continue;
            if (v == null) v = x;
            else if (!v.equals(x))
                throw new UnsupportedOperationException("the operator's functions read different values from one "
                        + "tuple; the GPU operator keeps one value per tuple");
        }
        return v != null ? v : 0;
    }

    private void bindEngine() {
        if (engine != null) return;
        List<Integer> kinds = new ArrayList<Integer>();
        StringBuilder sig = new StringBuilder().append(valueType).append('|').append(latenessSet ? maxLateness : "d");
        for (long[] w : windows) sig.append("|w").append(w[0]).append(',').append(w[1]).append(',').append(w[2])
                .append(',').append(w[3]);
        for (NativeFunctions.Binding b : bindings) {
            kinds.add(b.kind);
            sig.append("|f").append(b.kind);
        }
        engine = KeyedEngine.forThread(sig.toString(), valueType, windows, kinds, maxLateness, latenessSet);
        id = engine.newId();
    }

    private void configuredAfterUse() {
        if (engine != null)
            throw new UnsupportedOperationException("a per-key operator of a keyed connector was reconfigured after "
                    + "its first tuple: the shared keyed engine holds one configuration for all keys");
    }

    private void flush() {
        if (buffered == 0) return;
        check(api.processElements(op, tsBuf, valBuf, buffered));
        buffered = 0;
    }

    private void allocate(long capacity) {
        ByteBuffer ts = ByteBuffer.allocateDirect((int) (8 * capacity)).order(ByteOrder.nativeOrder());
        ByteBuffer vals = ByteBuffer.allocateDirect((int) (width * capacity)).order(ByteOrder.nativeOrder());
        if (buffered > 0) {
            NativeValues.copyPrefix(tsBuf, ts, (int) (8 * buffered));
            NativeValues.copyPrefix(valBuf, vals, (int) (width * buffered));
        }
        tsBuf = ts;
        valBuf = vals;
    }

    private int check(int rc) {
        if (rc >= 0) return rc;  // 1 = SCOTTY_WARN_LATE_DROPPED: tuples the reference drops too
        String msg = api.lastError(op);
        if (rc == ERR_INDEX) throw new IndexOutOfBoundsException(msg);  // the reference's exception type
        throw new UnsupportedOperationException(msg);
    }
}
