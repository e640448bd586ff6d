package de.tub.dima.scotty.slicing;

import java.lang.ref.WeakReference;
import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.ArrayList;
import java.util.Arrays;
import java.util.Collections;
import java.util.HashMap;
import java.util.HashSet;
import java.util.List;
import java.util.Map;
import java.util.Set;

/**
 * One keyed native operator behind all per-key {@link SlicingWindowOperator} instances of a keyed connector on one
 * task thread -- the drop-in at 1 M keys with the connectors unchanged.  Java 8 source.
 *
 * <p>The keyed connectors keep one SlicingWindowOperator per key in a HashMap, feed each tuple to its key's
 * operator and, when the watermark advances, call processWatermark(wm) on every key's operator in a loop
 * (F/KeyedScottyWindowOperator.java:56-86; the Samza, Kafka Streams, Storm, Spark and Beam connectors do the same).
 * One native operator per key would mean a million device allocations and a million watermark calls; instead every
 * instance gets a dense id (the uint32 key of ONE keyed native op, {@code SCOTTY_FLAG_KEYED}), its tuples go into
 * one off-heap (id, ts, value) micro-batch, and the first processWatermark(wm) of a round pushes the whole batch
 * (scotty_process_keyed_elements) and runs ONE native watermark over all keys; its rows come back grouped by key and
 * every instance's call is served from them.  Semantics per instance are the reference's: the native op runs an
 * independent SlicingWindowOperator per key (created on first sight, like the connector's HashMap).
 *
 * <p>Which instances join an engine (first match wins):
 * <ol>
 *   <li>explicitly: {@link SlicingWindowOperator#perKey} constructs a per-key instance, and
 *       {@link SlicingWindowOperator#keyedScope()} makes every operator constructed on the thread until the scope
 *       closes one (for a keyed wrapper the shim cannot recognise);</li>
 *   <li>by system property {@code scotty.keyed.engine}: {@code on} (every operator of the JVM is per-key),
 *       {@code off} (none is);</li>
 *   <li>otherwise ({@code auto}, the default) by caller: the constructing thread's stack holds one of
 *       {@link #KEYED_CONNECTORS} or of the comma-separated class names in system property
 *       {@code scotty.keyed.callers} (a user-written keyed wrapper names itself there).  The whole stack is
 *       searched, so a deeper call chain inside a connector is recognised; the matching frame is remembered per
 *       thread, so the next key's construction from the same call site is one array read, not a walk.</li>
 * </ol>
 *
 * <p>Instances share an engine only when their configuration (windows, functions, lateness, value type) is equal;
 * the connectors build every per-key operator identically, so one engine per connector per thread results.  Rows
 * of an instance that is not asked in a round (a caller that watermarks only some keys) wait for its next call,
 * ahead of that call's own rows, as the key's own operator would emit them then.  Ids are never reused (the
 * reference's map never evicts keys either).
 */
final class KeyedEngine {

    /** The reference's keyed connectors: a SlicingWindowOperator constructed from one of them joins an engine. */
    static final Set<String> KEYED_CONNECTORS = Collections.unmodifiableSet(new HashSet<String>(Arrays.asList(
            "de.tub.dima.scotty.flinkconnector.KeyedScottyWindowOperator",
            "de.tub.dima.scotty.samzaconnector.KeyedScottyWindowOperator",
            "de.tub.dima.scotty.kafkastreamsconnector.KeyedScottyWindowOperator",
            "de.tub.dima.scotty.stormconnector.KeyedScottyWindowOperator",
            "de.tub.dima.scotty.sparkconnector.KeyedScottyWindowOperator",
            "de.tub.dima.scotty.beamconnector.KeyedScottyWindowOperator")));

    /** Open {@link SlicingWindowOperator#keyedScope()} scopes of the thread (nesting depth). */
    static final ThreadLocal<int[]> SCOPE = new ThreadLocal<int[]>() {
        @Override
        protected int[] initialValue() {
            return new int[1];
        }
    };

    /** Whether an operator constructed now (not through perKey) is a per-key instance; see the class comment. */
    @SuppressWarnings("unchecked")
    static boolean sharedForCaller() {
        if (SCOPE.get()[0] > 0) return true;
        String mode = System.getProperty("scotty.keyed.engine", "auto");
        if (mode.equals("on")) return true;
        if (mode.equals("off")) return false;
        Set<String> callers = callerSet();
        Class<?>[] ctx = CallStack.classes();
        if (ctx == null) {  // no class context available: the stack trace (slower, same answer)
            for (StackTraceElement f : Thread.currentThread().getStackTrace())
                if (callers.contains(f.getClassName())) return true;
            return false;
        }
        // a keyed connector builds every key's operator from the same call site: the frame that matched last time on
        // this thread, at the same depth, answers at once (one array read instead of a walk per key at 1 M keys)
        // The hit is kept with the caller set it matched (a changed scotty.keyed.callers invalidates it) and holds the
        // class weakly (a pooled task thread must not pin a redeployed job's class loader).
        Object[] last = LAST_HIT.get();
        if (last[0] != null && last[2] == callers) {
            Class<?> hit = ((WeakReference<Class<?>>) last[0]).get();
            int d = (Integer) last[1];
            if (hit != null && d < ctx.length && ctx[d] == hit) return true;
        }
        for (int i = 0; i < ctx.length; i++) {
            if (callers.contains(ctx[i].getName())) {
                last[0] = new WeakReference<Class<?>>(ctx[i]);
                last[1] = i;
                last[2] = callers;
                return true;
            }
        }
        return false;
    }

    /** KEYED_CONNECTORS plus {@code scotty.keyed.callers}, parsed once per distinct property value. */
    private static volatile Object[] callerCache = {null, KEYED_CONNECTORS};

    @SuppressWarnings("unchecked")
    private static Set<String> callerSet() {
        String extra = System.getProperty("scotty.keyed.callers", "");
        Object[] c = callerCache;
        if (extra.equals(c[0])) return (Set<String>) c[1];
        Set<String> callers = KEYED_CONNECTORS;
        if (!extra.isEmpty()) {
            callers = new HashSet<String>(KEYED_CONNECTORS);
            for (String x : extra.split(",")) if (!x.trim().isEmpty()) callers.add(x.trim());
            callers = Collections.unmodifiableSet(callers);
        }
        callerCache = new Object[]{extra, callers};
        return callers;
    }

    /** {weak class, depth, caller set} of the stack frame that made the thread's last construction a per-key one. */
    private static final ThreadLocal<Object[]> LAST_HIT = new ThreadLocal<Object[]>() {
        @Override
        protected Object[] initialValue() {
            return new Object[3];
        }
    };

    /** The calling thread's classes, innermost first, without building StackTraceElements (Java 8 API). */
    private static final class CallStack extends SecurityManager {
        private static final CallStack INSTANCE = create();

        private static CallStack create() {
            try {
                return new CallStack();
            } catch (RuntimeException e) {  // an installed security manager may refuse: fall back to stack traces
                return null;
            }
        }

        static Class<?>[] classes() {
            return INSTANCE != null ? INSTANCE.getClassContext() : null;
        }
    }

    private static final ThreadLocal<Map<String, KeyedEngine>> ENGINES = new ThreadLocal<Map<String, KeyedEngine>>() {
        @Override
        protected Map<String, KeyedEngine> initialValue() {
            return new HashMap<String, KeyedEngine>();
        }
    };

    /** The engine of the calling thread for one configuration signature (created and configured on first use). */
    static KeyedEngine forThread(String signature, int valueType, List<long[]> windows, List<Integer> kinds,
                                 long maxLateness, boolean latenessSet) {
        Map<String, KeyedEngine> m = ENGINES.get();
        KeyedEngine e = m.get(signature);
        if (e == null) {
            e = new KeyedEngine(valueType, windows, kinds, maxLateness, latenessSet);
            m.put(signature, e);
        }
        return e;
    }

    /** One emitted window of one instance, before its function objects are rebuilt. */
    static final class Row {
        final long start, end;
        final int measure;
        final boolean has;
        final long[] words;

        Row(long start, long end, int measure, boolean has, long[] words) {
            this.start = start;
            this.end = end;
            this.measure = measure;
            this.has = has;
            this.words = words;
        }
    }

    private final NativeApi api = NativeApi.get();
    private final long op;
    private final int valueType, width;
    private int nextId = 0;
    private ByteBuffer keys, ts, vals;
    private long n = 0;
    private long roundWm = Long.MIN_VALUE;
    private boolean roundDone = false;
    private final Map<Integer, List<Row>> pending = new HashMap<Integer, List<Row>>();

    private KeyedEngine(int valueType, List<long[]> windows, List<Integer> kinds, long maxLateness,
                        boolean latenessSet) {
        this.valueType = valueType;
        this.width = valueType == NativeValues.VALUE_I32 ? 4 : 8;
        this.op = api.create(0, valueType, SlicingWindowOperator.FLAG_KEYED);
        for (long[] w : windows) check(api.addWindow(op, (int) w[0], (int) w[1], w[2], w[3]));
        for (int k : kinds) check(api.addAggregation(op, k));
        if (latenessSet) check(api.setMaxLateness(op, maxLateness));
        allocate(1 << 16);
    }

    int newId() {
        return nextId++;
    }

    /** processElement of instance {@code id}: appended to the round's micro-batch. */
    void add(int id, long t, Number value) {
        if (n == ts.capacity() / 8) allocate(2 * n);
        keys.putInt((int) (4 * n), id);
        ts.putLong((int) (8 * n), t);
        if (valueType == NativeValues.VALUE_I32) vals.putInt((int) (4 * n), value.intValue());
        else if (valueType == NativeValues.VALUE_I64) vals.putLong((int) (8 * n), value.longValue());
        else vals.putDouble((int) (8 * n), value.doubleValue());
        n++;
    }

    /** processWatermark(wm) of instance {@code id}: the round's rows of that instance. */
    List<Row> watermark(int id, long wm) {
        flush();
        if (!roundDone || wm != roundWm) {  // the round's first call: one watermark over every key
            NativeApi.Windows w = new NativeApi.Windows();
            int rc = api.processWatermark(op, wm, w);
            if (rc == SlicingWindowOperator.ERR_INDEX) throw new IndexOutOfBoundsException(api.lastError(op));
            check(rc);
            for (int i = 0; i < w.n; i++) {
                long[] words = new long[w.values.length];
                for (int k = 0; k < words.length; k++) words[k] = w.values[k][i];
                List<Row> rows = pending.get(w.key[i]);
                if (rows == null) {
                    rows = new ArrayList<Row>();
                    pending.put(w.key[i], rows);
                }
                rows.add(new Row(w.start[i], w.end[i], w.measure[i], w.has[i] != 0, words));
            }
            roundWm = wm;
            roundDone = true;
        }
        List<Row> r = pending.remove(id);
        return r != null ? r : Collections.<Row>emptyList();
    }

    private void flush() {
        if (n == 0) return;
        check(api.processKeyedElements(op, keys, ts, vals, n));
        n = 0;
        // tuples after a round: the next call runs a new native watermark, as every key's own operator would on
        // its next processWatermark (the connectors call it only when the watermark advanced)
        roundDone = false;
    }

    private void allocate(long capacity) {
        ByteBuffer k = ByteBuffer.allocateDirect((int) (4 * capacity)).order(ByteOrder.nativeOrder());
        ByteBuffer t = ByteBuffer.allocateDirect((int) (8 * capacity)).order(ByteOrder.nativeOrder());
        ByteBuffer v = ByteBuffer.allocateDirect((int) (width * capacity)).order(ByteOrder.nativeOrder());
        if (n > 0) {
            NativeValues.copyPrefix(keys, k, (int) (4 * n));
            NativeValues.copyPrefix(ts, t, (int) (8 * n));
            NativeValues.copyPrefix(vals, v, (int) (width * n));
        }
        keys = k;
        ts = t;
        vals = v;
    }

    private void check(int rc) {
        if (rc >= 0) return;
        throw new UnsupportedOperationException(api.lastError(op));
    }
}
