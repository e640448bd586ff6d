package de.tub.dima.scotty.slicing;

import java.nio.ByteBuffer;

/**
 * The C-ABI of include/scotty_mi355x.h as the shim calls it.  Java 8 source.  Two bindings implement it:
 * {@link JniApi} (JNI through {@code java/jni/scotty_jni.c}; the default, any JDK from 8 -- the reference's target,
 * pom.xml:50) and {@code FfmApi} (the Java 22 Foreign Function and Memory API, no glue library; an optional source
 * set, {@code java/ffm}, compiled only for JDK 22+).  Tuple buffers are direct ByteBuffers (off-heap, native byte
 * order), which both bindings hand to the library without a copy.  Selection: system property
 * {@code scotty.native.binding} = {@code jni} (default) | {@code ffm} (fails loudly when the FFM class or runtime is
 * absent).
 */
interface NativeApi {

    /** One processWatermark result (scotty_windows), copied into Java arrays. */
    final class Windows {
        int n;
        long[] start, end;
        int[] measure;
        byte[] has;
        long[][] values;   // [n_aggs][n]
        int[] key;         // keyed ops: the uint32 key (dense instance id) of every row; null otherwise
    }

    /** scotty_create; returns the op handle, throws on error. */
    long create(int device, int valueType, int flags);

    void destroy(long op);

    String lastError(long op);

    int addWindow(long op, int kind, int measure, long a, long b);

    int addAggregation(long op, int kind);

    int setMaxLateness(long op, long maxLateness);

    /** scotty_process_elements: n tuples, ts = int64[n], val = n values of the op's value type (direct buffers). */
    int processElements(long op, ByteBuffer ts, ByteBuffer val, long n);

    /** scotty_process_keyed_elements: key = uint32[n]. */
    int processKeyedElements(long op, ByteBuffer key, ByteBuffer ts, ByteBuffer val, long n);

    /** scotty_process_watermark, the columns copied into {@code out}. */
    int processWatermark(long op, long watermark, Windows out);

    /**
     * scotty_first_indices: the arrival indices a later window can still return as its first partial's tuple
     * (SCOTTY_AGG_FIRST operators), ascending; null on error (lastError has the message).
     */
    long[] firstIndices(long op);

    /** The binding of this JVM (see the class comment). */
    static NativeApi get() {
        return Holder.API;
    }

    final class Holder {
        static final NativeApi API = select();

        private static NativeApi select() {
            String b = System.getProperty("scotty.native.binding", "jni");
            if (b.equals("ffm")) {
                try {
                    // by name: the main source set compiles and runs on Java 8, without java.lang.foreign
                    Class.forName("java.lang.foreign.Linker");
                    return (NativeApi) Class.forName("de.tub.dima.scotty.slicing.FfmApi").getDeclaredConstructor()
                            .newInstance();
                } catch (ReflectiveOperationException e) {
                    throw new UnsupportedOperationException("FFM binding unavailable (JDK 22+ and the java/ffm source "
                            + "set are needed)", e);
                } catch (LinkageError e) {
                    throw new UnsupportedOperationException("FFM binding unavailable (JDK 22+ and the java/ffm source "
                            + "set are needed)", e);
                }
            }
            if (!b.equals("jni"))
                throw new UnsupportedOperationException("scotty.native.binding must be jni or ffm, not " + b);
            return new JniApi();
        }
    }
}
