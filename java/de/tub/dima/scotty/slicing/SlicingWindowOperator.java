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

import java.lang.foreign.Arena;
import java.lang.foreign.FunctionDescriptor;
import java.lang.foreign.Linker;
import java.lang.foreign.MemorySegment;
import java.lang.foreign.SymbolLookup;
import java.lang.invoke.MethodHandle;
import java.util.ArrayList;
import java.util.List;

import static java.lang.foreign.ValueLayout.ADDRESS;
import static java.lang.foreign.ValueLayout.JAVA_BYTE;
import static java.lang.foreign.ValueLayout.JAVA_DOUBLE;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;

/**
 * Drop-in for the reference's {@code de.tub.dima.scotty.slicing.SlicingWindowOperator}
 * (slicing/src/main/java/de/tub/dima/scotty/slicing/SlicingWindowOperator.java:20-70), backed by
 * {@code libscotty_mi355x.so} through the Java 22 Foreign Function and Memory API: one native operator per
 * instance, the C-ABI of {@code include/scotty_mi355x.h}.  Put this class ahead of the reference's slicing jar
 * on the classpath; the connectors' {@code new SlicingWindowOperator<>(stateFactory)} then binds here.
 *
 * <p>processElement buffers the tuple off-heap (no native call); the buffer goes to the GPU as one micro-batch
 * (scotty_process_elements) before the next processWatermark or configuration call, which is where the reference's
 * per-tuple work becomes observable.  Window results come back as SoA columns (scotty_windows) and are boxed into
 * {@link NativeAggregateWindow}s in the reference's emission order.
 *
 * <p>Only aggregations with a GPU kind run ({@link NativeValues#kindOf}); anything else is rejected with
 * UnsupportedOperationException at addAggregation -- there is no CPU fallback.
 */
public class SlicingWindowOperator<InputType> implements WindowOperator<InputType> {

    private static final Linker LINKER = Linker.nativeLinker();
    private static final SymbolLookup LIB = SymbolLookup.libraryLookup(
            System.getProperty("scotty.native.lib", "libscotty_mi355x.so"), Arena.global());

    private static MethodHandle handle(String name, FunctionDescriptor d) {
        return LINKER.downcallHandle(LIB.find(name).orElseThrow(() -> new UnsatisfiedLinkError(name)), d);
    }

    // include/scotty_mi355x.h
    private static final MethodHandle CREATE = handle("scotty_create",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT, JAVA_INT));
    private static final MethodHandle DESTROY = handle("scotty_destroy", FunctionDescriptor.ofVoid(ADDRESS));
    private static final MethodHandle LAST_ERROR = handle("scotty_last_error", FunctionDescriptor.of(ADDRESS, ADDRESS));
    private static final MethodHandle ADD_WINDOW = handle("scotty_add_window",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT, JAVA_LONG, JAVA_LONG));
    private static final MethodHandle ADD_AGGREGATION = handle("scotty_add_aggregation",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_INT));
    private static final MethodHandle SET_MAX_LATENESS = handle("scotty_set_max_lateness",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_LONG));
    private static final MethodHandle PROCESS_ELEMENTS = handle("scotty_process_elements",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS, JAVA_LONG));
    private static final MethodHandle PROCESS_WATERMARK = handle("scotty_process_watermark",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_LONG, ADDRESS));

    // SCOTTY_WIN_* / SCOTTY_MEASURE_* / SCOTTY_VALUE_* / error codes
    private static final int WIN_TUMBLING = 0, WIN_SLIDING = 1, WIN_SESSION = 2, WIN_FIXED_BAND = 3;
    private static final int ERR_INDEX = -5;

    // scotty_windows: size_t n_windows; int32 n_aggs (+4 pad); start, end, measure, has_value; values[8]; key
    private static final long RES_BYTES = 120, OFF_N = 0, OFF_START = 16, OFF_END = 24, OFF_MEASURE = 32,
            OFF_HAS = 40, OFF_VALUES = 48;

    // native state: created in the constructor on the task that runs the operator (connectors build operators in
    // open(), not by deserialization), so it is not part of the serialized form
    private final transient Arena arena = Arena.ofShared();
    private final transient MemorySegment op;
    private final int valueType;
    private final NativeValues.Extractor<InputType> extractor;
    private final List<Integer> kinds = new ArrayList<>();
    private transient MemorySegment tsBuf, valBuf;
    private long buffered = 0;

    /** S/SlicingWindowOperator.java:30-37: the state factory is not used (slices live in HBM). */
    public SlicingWindowOperator(StateFactory stateFactory) {
        this(stateFactory, NativeValues.VALUE_I32, NativeValues.defaultExtractor());
    }

    /** valueType: NativeValues.VALUE_I32 / VALUE_I64 / VALUE_F64; extractor: the numeric value of a tuple. */
    public SlicingWindowOperator(StateFactory stateFactory, int valueType, NativeValues.Extractor<InputType> extractor) {
        this.valueType = valueType;
        this.extractor = extractor;
        MemorySegment out = arena.allocate(ADDRESS);
        check(callInt(CREATE, out, 0, valueType, 0));
        this.op = out.get(ADDRESS, 0);
        allocate(1 << 16);
    }

    @Override
    public void processElement(InputType element, long ts) {
        if (buffered == tsBuf.byteSize() / 8) allocate(2 * buffered);
        tsBuf.setAtIndex(JAVA_LONG, buffered, ts);
        if (valueType == NativeValues.VALUE_I32) valBuf.setAtIndex(JAVA_INT, buffered, (int) extractor.value(element));
        else if (valueType == NativeValues.VALUE_I64) valBuf.setAtIndex(JAVA_LONG, buffered, extractor.value(element));
        else valBuf.setAtIndex(JAVA_DOUBLE, buffered, extractor.doubleValue(element));
        buffered++;
    }

    /** S/SlicingWindowOperator.java:46-49 (WindowManager.processWatermark, S/WindowManager.java:38-61). */
    @Override
    public List<AggregateWindow> processWatermark(long watermarkTs) {
        flush();
        MemorySegment res = arena.allocate(RES_BYTES, 8);
        check(callInt(PROCESS_WATERMARK, op, watermarkTs, res));
        long n = res.get(JAVA_LONG, OFF_N);
        List<AggregateWindow> windows = new ArrayList<>((int) n);
        if (n == 0) return windows;
        MemorySegment start = res.get(ADDRESS, OFF_START).reinterpret(8 * n);
        MemorySegment end = res.get(ADDRESS, OFF_END).reinterpret(8 * n);
        MemorySegment measure = res.get(ADDRESS, OFF_MEASURE).reinterpret(4 * n);
        MemorySegment has = res.get(ADDRESS, OFF_HAS).reinterpret(n);
        MemorySegment[] values = new MemorySegment[kinds.size()];
        for (int k = 0; k < values.length; k++) values[k] = res.get(ADDRESS, OFF_VALUES + 8L * k).reinterpret(8 * n);
        for (long i = 0; i < n; i++) {
            List<Object> agg = new ArrayList<>(values.length);
            boolean hasValue = has.get(JAVA_BYTE, i) != 0;
            if (hasValue)
                for (int k = 0; k < values.length; k++)
                    agg.add(NativeValues.box(kinds.get(k), values[k].getAtIndex(JAVA_LONG, i)));
            windows.add(new NativeAggregateWindow(
                    measure.getAtIndex(JAVA_INT, i) == 0 ? WindowMeasure.Time : WindowMeasure.Count,
                    start.getAtIndex(JAVA_LONG, i), end.getAtIndex(JAVA_LONG, i), hasValue, agg));
        }
        return windows;
    }

    /** WindowManager.addWindowAssigner (S/WindowManager.java:121-147). */
    @Override
    public void addWindowAssigner(Window window) {
        flush();
        int m = window.getWindowMeasure() == WindowMeasure.Time ? 0 : 1;
        if (window instanceof TumblingWindow t) {
            check(callInt(ADD_WINDOW, op, WIN_TUMBLING, m, t.getSize(), 0L));
        } else if (window instanceof SlidingWindow s) {
            check(callInt(ADD_WINDOW, op, WIN_SLIDING, m, s.getSize(), s.getSlide()));
        } else if (window instanceof SessionWindow s) {
            check(callInt(ADD_WINDOW, op, WIN_SESSION, m, s.getGap(), 0L));
        } else if (window instanceof FixedBandWindow f) {
            check(callInt(ADD_WINDOW, op, WIN_FIXED_BAND, m, f.getStart(), f.getSize()));
        } else {
            throw new UnsupportedOperationException("window type without a GPU kind: " + window);
        }
    }

    /** WindowManager.addAggregation (S/WindowManager.java:196-198). */
    @Override
    public <OutputType> void addAggregation(AggregateFunction<InputType, ?, OutputType> windowFunction) {
        flush();
        int kind = NativeValues.kindOf(windowFunction, valueType);
        if (kind < 0)
            throw new UnsupportedOperationException("AggregateFunction without a GPU kind (user lambdas cannot run on "
                    + "the GPU): " + windowFunction.getClass().getName());
        check(callInt(ADD_AGGREGATION, op, kind));
        kinds.add(kind & 0xFFFF);
    }

    /** S/SlicingWindowOperator.java:57-63. */
    public <Agg, OutputType> void addWindowFunction(AggregateFunction<InputType, Agg, OutputType> windowFunction) {
        addAggregation(windowFunction);
    }

    @Override
    public void setMaxLateness(long maxLateness) {
        flush();
        check(callInt(SET_MAX_LATENESS, op, maxLateness));
    }

    /** Frees the native operator (the reference's operator is garbage collected; here HBM is released). */
    public void close() {
        try {
            DESTROY.invokeExact(op);
        } catch (Throwable t) {
            throw new RuntimeException(t);
        }
        arena.close();
    }

    private void flush() {
        if (buffered == 0) return;
        check(callInt(PROCESS_ELEMENTS, op, tsBuf, valBuf, buffered));
        buffered = 0;
    }

    private void allocate(long capacity) {
        long width = valueType == NativeValues.VALUE_I32 ? 4 : 8;
        MemorySegment ts = arena.allocate(8 * capacity, 8), vals = arena.allocate(width * capacity, 8);
        if (buffered > 0) {
            MemorySegment.copy(tsBuf, 0, ts, 0, 8 * buffered);
            MemorySegment.copy(valBuf, 0, vals, 0, width * buffered);
        }
        tsBuf = ts;
        valBuf = vals;
    }

    private void check(int rc) {
        if (rc >= 0) return;  // 1 = SCOTTY_WARN_LATE_DROPPED: tuples the reference drops too
        String msg;
        try {
            msg = ((MemorySegment) LAST_ERROR.invoke(op)).reinterpret(4096).getString(0);
        } catch (Throwable t) {
            msg = "scotty error " + rc;
        }
        if (rc == ERR_INDEX) throw new IndexOutOfBoundsException(msg);  // the reference's exception type
        throw new UnsupportedOperationException(msg);
    }

    private static int callInt(MethodHandle mh, Object... args) {
        try {
            return (int) mh.invokeWithArguments(args);
        } catch (Throwable t) {
            throw new RuntimeException(t);
        }
    }
}
