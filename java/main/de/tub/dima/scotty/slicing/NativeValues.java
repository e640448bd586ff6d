package de.tub.dima.scotty.slicing;

import java.io.Serializable;
import java.nio.ByteBuffer;

/**
 * Constants of include/scotty_mi355x.h (value types, SCOTTY_AGG_* function kinds), the user-facing {@link NativeKind}
 * interface, tuple value extractors and the boxing of lowered int64 result words.  Java 8 source.  Which reference functions map to
 * which kind is decided in {@link NativeFunctions} (explicit, by fully-qualified class name or {@link NativeKind}).
 */
public final class NativeValues {

    public static final int VALUE_I32 = 0, VALUE_I64 = 1, VALUE_F64 = 2;

    public static final int AGG_SUM_I32 = 0, AGG_COUNT = 1, AGG_MIN_I32 = 2, AGG_MAX_I32 = 3, AGG_SUM_I64 = 4,
            AGG_MIN_I64 = 5, AGG_MAX_I64 = 6, AGG_SUM_F64 = 7, AGG_MIN_F64 = 8, AGG_MAX_F64 = 9;
    /** SCOTTY_AGG_FIRST: the arrival index of the window's first partial's tuple (registered by the shim itself). */
    public static final int AGG_FIRST = 10;
    public static final int AGG_INVERTIBLE = 0x10000;

    private NativeValues() {
    }

    /**
     * A user function that states the GPU kind (SCOTTY_AGG_*) its lift / combine / lower compute, the number its lift
     * reads from a tuple, and how the lowered number becomes the object its {@code lower()} returns.  The defaults
     * read a {@link Number} tuple and return the boxed number ({@link #box}).
     */
    public interface NativeKind<InputType> {
        int scottyKind();

        /** The argument of lift as a number (int/long kinds: {@code longValue}, double kinds: {@code doubleValue}). */
        default Number scottyValue(InputType tuple) {
            if (tuple instanceof Number) return (Number) tuple;
            throw new IllegalArgumentException("NativeKind function on a non-numeric tuple " + tuple
                    + ": override scottyValue");
        }

        /**
         * The reference's lower() result for the lowered number {@code boxed} ({@link #box} of the result word) of a
         * window; {@code exemplar} is a tuple of this operator instance (e.g. to copy a key field).
         */
        default Object scottyRebuild(Object boxed, InputType exemplar) {
            return boxed;
        }
    }

    /** The numeric value a tuple contributes (the argument of the function's lift). */
    public interface Extractor<T> extends Serializable {
        long value(T tuple);

        default double doubleValue(T tuple) {
            return value(tuple);
        }
    }

    /** Numbers as themselves; anything else needs a function binding or an explicit Extractor. */
    public static <T> Extractor<T> numberExtractor() {
        return new Extractor<T>() {
            @Override
            public long value(T tuple) {
                return number(tuple).longValue();
            }

            @Override
            public double doubleValue(T tuple) {
                return number(tuple).doubleValue();
            }
        };
    }

    static Number number(Object tuple) {
        if (tuple instanceof Number) return (Number) tuple;
        throw new IllegalArgumentException("no numeric value in tuple " + tuple
                + ": register a function NativeFunctions knows, implement NativeKind.scottyValue, or pass an Extractor");
    }

    /** Boxes one lowered result word as the kind's Java type (Integer, Long or Double). */
    public static Object box(int kind, long bits) {
        switch (kind & 0xFFFF) {
            case AGG_SUM_I32:
            case AGG_COUNT:
            case AGG_MIN_I32:
            case AGG_MAX_I32:
                return (int) bits;
            case AGG_SUM_I64:
            case AGG_MIN_I64:
            case AGG_MAX_I64:
                return bits;
            default:
                return Double.longBitsToDouble(bits);
        }
    }

    /** Copies the first {@code bytes} of {@code src} to the start of {@code dst} (positions of both untouched). */
    static void copyPrefix(ByteBuffer src, ByteBuffer dst, int bytes) {
        ByteBuffer from = src.duplicate();
        from.position(0);
        from.limit(bytes);
        ByteBuffer to = dst.duplicate();
        to.position(0);
        to.put(from);
    }
}
