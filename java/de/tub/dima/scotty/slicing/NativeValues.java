package de.tub.dima.scotty.slicing;

import de.tub.dima.scotty.core.windowFunction.AggregateFunction;
import de.tub.dima.scotty.core.windowFunction.InvertibleAggregateFunction;

import java.io.Serializable;
import java.lang.reflect.Field;

/**
 * Mapping between the reference's aggregate functions and the GPU's function kinds (SCOTTY_AGG_* of
 * include/scotty_mi355x.h), the numeric value of a tuple, and the boxing of lowered result columns.
 *
 * <p>A function has a GPU kind when (1) it implements {@link NativeKind} (the user states which kind its
 * lift / combine / lower compute), or (2) it is one of the functions the reference ships for these semantics:
 * benchmark {@code SumAggregation} and the demos' {@code Sum} / {@code SumWindowFunction} (Integer sum, int32
 * wrap), {@code Count} (lift 1, combine +), {@code Min} / {@code MinWindowFunction} (Math.min),
 * {@code Max} / {@code MaxWindowFunction} (Math.max).  An {@link InvertibleAggregateFunction} adds
 * SCOTTY_AGG_INVERTIBLE (LazySlice record removal by invert instead of recompute, S/state/AggregateValueState.java:
 * 33-49).  Anything else -- user lambdas, quantiles -- has no kind (-1): the operator rejects it loudly.
 */
public final class NativeValues {

    public static final int VALUE_I32 = 0, VALUE_I64 = 1, VALUE_F64 = 2;

    public static final int AGG_SUM_I32 = 0, AGG_COUNT = 1, AGG_MIN_I32 = 2, AGG_MAX_I32 = 3, AGG_SUM_I64 = 4,
            AGG_MIN_I64 = 5, AGG_MAX_I64 = 6, AGG_SUM_F64 = 7, AGG_MIN_F64 = 8, AGG_MAX_F64 = 9;
    public static final int AGG_INVERTIBLE = 0x10000;

    private NativeValues() {
    }

    /** A user function that states its GPU kind (SCOTTY_AGG_*). */
    public interface NativeKind {
        int scottyKind();
    }

    /** The numeric value a tuple contributes (the argument of the function's lift). */
    public interface Extractor<T> extends Serializable {
        long value(T tuple);

        default double doubleValue(T tuple) {
            return value(tuple);
        }
    }

    /**
     * Numbers as themselves; otherwise the tuple's public field {@code f1} (the Flink Tuple2 value field the
     * reference's demo functions lift, e.g. D/flink-demo/.../SumWindowFunction.java).
     */
    public static <T> Extractor<T> defaultExtractor() {
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

    private static Number number(Object tuple) {
        if (tuple instanceof Number n) return n;
        try {
            Field f = tuple.getClass().getField("f1");
            Object v = f.get(tuple);
            if (v instanceof Number n) return n;
        } catch (ReflectiveOperationException ignored) {
            // fall through
        }
        throw new IllegalArgumentException("no numeric value in tuple " + tuple + ": pass an Extractor");
    }

    /** SCOTTY_AGG_* kind of a function for an operator of the given value type, or -1. */
    public static int kindOf(AggregateFunction<?, ?, ?> fn, int valueType) {
        int kind;
        if (fn instanceof NativeKind k) {
            kind = k.scottyKind();
        } else {
            String name = fn.getClass().getSimpleName();
            int sum = valueType == VALUE_I32 ? AGG_SUM_I32 : valueType == VALUE_I64 ? AGG_SUM_I64 : AGG_SUM_F64;
            int min = valueType == VALUE_I32 ? AGG_MIN_I32 : valueType == VALUE_I64 ? AGG_MIN_I64 : AGG_MIN_F64;
            int max = valueType == VALUE_I32 ? AGG_MAX_I32 : valueType == VALUE_I64 ? AGG_MAX_I64 : AGG_MAX_F64;
            switch (name) {
                case "SumAggregation", "Sum", "SumWindowFunction" -> kind = sum;
                case "Count" -> kind = AGG_COUNT;
                case "Min", "MinWindowFunction" -> kind = min;
                case "Max", "MaxWindowFunction" -> kind = max;
                default -> kind = -1;
            }
        }
        if (kind < 0) return -1;
        return fn instanceof InvertibleAggregateFunction ? kind | AGG_INVERTIBLE : kind;
    }

    /** Boxes one lowered result (int64 column cell) as the reference's lower() would return it. */
    public static Object box(int kind, long bits) {
        switch (kind & 0xFFFF) {
            case AGG_SUM_I32, AGG_COUNT, AGG_MIN_I32, AGG_MAX_I32:
                return (int) bits;
            case AGG_SUM_I64, AGG_MIN_I64, AGG_MAX_I64:
                return bits;
            default:
                return Double.longBitsToDouble(bits);
        }
    }
}
