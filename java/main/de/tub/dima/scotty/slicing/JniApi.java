package de.tub.dima.scotty.slicing;

import java.nio.ByteBuffer;

/**
 * JNI binding of the C-ABI ({@code java/jni/scotty_jni.c} -> {@code libscotty_jni.so}, linked against
 * {@code libscotty_mi355x.so}).  Every native method is a thin forward to one scotty_* call; tuple buffers are
 * direct ByteBuffers (GetDirectBufferAddress, no copy); processWatermark copies the result columns into new Java
 * arrays.  Library name: system property {@code scotty.jni.lib} (default {@code scotty_jni}).  The default binding;
 * Java 8 source.
 */
final class JniApi implements NativeApi {

    static {
        System.loadLibrary(System.getProperty("scotty.jni.lib", "scotty_jni"));
    }

    private static native long create0(int device, int valueType, int flags, int[] rc);

    private static native void destroy0(long op);

    private static native String lastError0(long op);

    private static native int addWindow0(long op, int kind, int measure, long a, long b);

    private static native int addAggregation0(long op, int kind);

    private static native int setMaxLateness0(long op, long maxLateness);

    private static native int processElements0(long op, ByteBuffer ts, ByteBuffer val, long n);

    private static native int processKeyedElements0(long op, ByteBuffer key, ByteBuffer ts, ByteBuffer val, long n);

    private static native int processWatermark0(long op, long watermark, Windows out);

    private static native long[] firstIndices0(long op);

    @Override
    public long create(int device, int valueType, int flags) {
        int[] rc = new int[1];
        long op = create0(device, valueType, flags, rc);
        if (rc[0] < 0 || op == 0) throw new UnsupportedOperationException("scotty_create failed: " + rc[0]);
        return op;
    }

    @Override
    public void destroy(long op) {
        destroy0(op);
    }

    @Override
    public String lastError(long op) {
        return lastError0(op);
    }

    @Override
    public int addWindow(long op, int kind, int measure, long a, long b) {
        return addWindow0(op, kind, measure, a, b);
    }

    @Override
    public int addAggregation(long op, int kind) {
        return addAggregation0(op, kind);
    }

    @Override
    public int setMaxLateness(long op, long maxLateness) {
        return setMaxLateness0(op, maxLateness);
    }

    @Override
    public int processElements(long op, ByteBuffer ts, ByteBuffer val, long n) {
        return processElements0(op, ts, val, n);
    }

    @Override
    public int processKeyedElements(long op, ByteBuffer key, ByteBuffer ts, ByteBuffer val, long n) {
        return processKeyedElements0(op, key, ts, val, n);
    }

    @Override
    public int processWatermark(long op, long watermark, Windows out) {
        return processWatermark0(op, watermark, out);
    }

    @Override
    public long[] firstIndices(long op) {
        return firstIndices0(op);
    }
}
