package de.tub.dima.scotty.slicing;

import java.lang.foreign.Arena;
import java.lang.foreign.FunctionDescriptor;
import java.lang.foreign.Linker;
import java.lang.foreign.MemorySegment;
import java.lang.foreign.SymbolLookup;
import java.lang.invoke.MethodHandle;
import java.nio.ByteBuffer;

import static java.lang.foreign.ValueLayout.ADDRESS;
import static java.lang.foreign.ValueLayout.JAVA_BYTE;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;

/**
 * Panama (Java 22 FFM) binding of the C-ABI -- the optional {@code java/ffm} source set, compiled only with JDK 22+ and
 * selected with {@code -Dscotty.native.binding=ffm} (JNI is the default, java/main/.../NativeApi.java): downcall handles on {@code libscotty_mi355x.so} (system property
 * {@code scotty.native.lib}), direct ByteBuffers passed as MemorySegment.ofBuffer (no copy), and the scotty_windows
 * result struct read from one reusable per-thread segment (no allocation per watermark).
 */
final class FfmApi implements NativeApi {

    private static final Linker LINKER = Linker.nativeLinker();
    private static final SymbolLookup LIB = SymbolLookup.libraryLookup(
            System.getProperty("scotty.native.lib", "libscotty_mi355x.so"), Arena.global());

    private static MethodHandle handle(String name, FunctionDescriptor d) {
        return LINKER.downcallHandle(LIB.find(name).orElseThrow(() -> new UnsatisfiedLinkError(name)), d);
    }

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
    private static final MethodHandle PROCESS_KEYED = handle("scotty_process_keyed_elements",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS, ADDRESS, JAVA_LONG));
    private static final MethodHandle PROCESS_WATERMARK = handle("scotty_process_watermark",
            FunctionDescriptor.of(JAVA_INT, ADDRESS, JAVA_LONG, ADDRESS));
    private static final MethodHandle FIRST_INDICES = handle("scotty_first_indices",
            FunctionDescriptor.of(JAVA_LONG, ADDRESS, ADDRESS, JAVA_LONG));

    // scotty_windows: size_t n_windows; int32 n_aggs (+4 pad); start, end, measure, has_value; values[8]; key
    private static final long RES_BYTES = 120, OFF_N = 0, OFF_NAGGS = 8, OFF_START = 16, OFF_END = 24,
            OFF_MEASURE = 32, OFF_HAS = 40, OFF_VALUES = 48, OFF_KEY = 112;

    // one result struct per thread, allocated once (a watermark allocates nothing native)
    private static final ThreadLocal<MemorySegment> RESULT =
            ThreadLocal.withInitial(() -> Arena.global().allocate(RES_BYTES, 8));

    private static MemorySegment ptr(long op) {
        return MemorySegment.ofAddress(op);
    }

    @Override
    public long create(int device, int valueType, int flags) {
        try (Arena a = Arena.ofConfined()) {
            MemorySegment out = a.allocate(ADDRESS);
            int rc = (int) CREATE.invokeExact(out, device, valueType, flags);
            if (rc < 0) throw new UnsupportedOperationException("scotty_create failed: " + rc);
            return out.get(ADDRESS, 0).address();
        } catch (RuntimeException e) {
            throw e;
        } catch (Throwable t) {
            throw new RuntimeException(t);
        }
    }

    @Override
    public void destroy(long op) {
        try {
            DESTROY.invokeExact(ptr(op));
        } catch (Throwable t) {
            throw new RuntimeException(t);
        }
    }

    @Override
    public String lastError(long op) {
        try {
            return ((MemorySegment) LAST_ERROR.invokeExact(ptr(op))).reinterpret(4096).getString(0);
        } catch (Throwable t) {
            return "scotty error";
        }
    }

    @Override
    public int addWindow(long op, int kind, int measure, long a, long b) {
        try {
            return (int) ADD_WINDOW.invokeExact(ptr(op), kind, measure, a, b);
        } catch (Throwable t) {
            throw new RuntimeException(t);
        }
    }

    @Override
    public int addAggregation(long op, int kind) {
        try {
            return (int) ADD_AGGREGATION.invokeExact(ptr(op), kind);
        } catch (Throwable t) {
            throw new RuntimeException(t);
        }
    }

    @Override
    public int setMaxLateness(long op, long maxLateness) {
        try {
            return (int) SET_MAX_LATENESS.invokeExact(ptr(op), maxLateness);
        } catch (Throwable t) {
            throw new RuntimeException(t);
        }
    }

    @Override
    public int processElements(long op, ByteBuffer ts, ByteBuffer val, long n) {
        try {
            return (int) PROCESS_ELEMENTS.invokeExact(ptr(op), MemorySegment.ofBuffer(ts), MemorySegment.ofBuffer(val), n);
        } catch (Throwable t) {
            throw new RuntimeException(t);
        }
    }

    @Override
    public int processKeyedElements(long op, ByteBuffer key, ByteBuffer ts, ByteBuffer val, long n) {
        try {
            return (int) PROCESS_KEYED.invokeExact(ptr(op), MemorySegment.ofBuffer(key), MemorySegment.ofBuffer(ts),
                    MemorySegment.ofBuffer(val), n);
        } catch (Throwable t) {
            throw new RuntimeException(t);
        }
    }

    @Override
    public int processWatermark(long op, long watermark, Windows out) {
        MemorySegment res = RESULT.get();
        int rc;
        try {
            rc = (int) PROCESS_WATERMARK.invokeExact(ptr(op), watermark, res);
        } catch (Throwable t) {
            throw new RuntimeException(t);
        }
        if (rc < 0) return rc;
        int n = (int) res.get(JAVA_LONG, OFF_N);
        int nAggs = res.get(JAVA_INT, OFF_NAGGS);
        out.n = n;
        out.start = column(res, OFF_START, n).toArray(JAVA_LONG);
        out.end = column(res, OFF_END, n).toArray(JAVA_LONG);
        out.measure = n == 0 ? new int[0] : res.get(ADDRESS, OFF_MEASURE).reinterpret(4L * n).toArray(JAVA_INT);
        out.has = n == 0 ? new byte[0] : res.get(ADDRESS, OFF_HAS).reinterpret(n).toArray(JAVA_BYTE);
        out.values = new long[nAggs][];
        for (int k = 0; k < nAggs; k++) out.values[k] = column(res, OFF_VALUES + 8L * k, n).toArray(JAVA_LONG);
        MemorySegment key = res.get(ADDRESS, OFF_KEY);
        out.key = key.address() == 0 || n == 0 ? null : key.reinterpret(4L * n).toArray(JAVA_INT);
        return rc;
    }

    @Override
    public long[] firstIndices(long op) {
        try {
            long n = (long) FIRST_INDICES.invokeExact(ptr(op), MemorySegment.NULL, 0L);
            if (n <= 0) return n < 0 ? null : new long[0];
            try (Arena a = Arena.ofConfined()) {
                MemorySegment buf = a.allocate(8L * n, 8);
                long m = (long) FIRST_INDICES.invokeExact(ptr(op), buf, n);
                return m == n ? buf.toArray(JAVA_LONG) : null;
            }
        } catch (Throwable t) {
            throw new RuntimeException(t);
        }
    }

    private static MemorySegment column(MemorySegment res, long off, int n) {
        return n == 0 ? MemorySegment.NULL : res.get(ADDRESS, off).reinterpret(8L * n);
    }
}
