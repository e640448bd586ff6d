package de.tub.dima.scotty.slicing;

import de.tub.dima.scotty.core.windowFunction.AggregateFunction;
import de.tub.dima.scotty.core.windowFunction.InvertibleAggregateFunction;

import java.lang.invoke.MethodHandle;
import java.lang.invoke.MethodHandles;
import java.lang.invoke.MethodType;
import java.lang.reflect.Constructor;
import java.lang.reflect.Method;
import java.util.Collections;
import java.util.HashMap;
import java.util.Map;
import java.util.Objects;

import static de.tub.dima.scotty.slicing.NativeValues.*;

/**
 * Which aggregate functions run on the GPU, and how their tuples and results cross the boundary.  Java 8 source.
 *
 * <p>A function runs on the GPU only if (1) it implements {@link NativeValues.NativeKind}, or (2) its
 * FULLY-QUALIFIED class name is one of the reference's own shipped functions listed in {@link #REGISTRY}, whose
 * lift / combine / lower this class restates (a user class that merely shares a simple name such as {@code Sum}
 * gets no kind).  Everything else -- user lambdas, quantiles -- is rejected with UnsupportedOperationException at
 * addAggregation: there is no CPU fallback and no silent guess.
 *
 * <p>Result objects are rebuilt as the reference's {@code lower()} returns them (ReduceAggregateFunction's lower is
 * the identity, C/windowFunction/ReduceAggregateFunction.java:13-15): the demos' Flink functions aggregate
 * {@code Tuple2<Integer,Integer>} and keep {@code partialAggregate1.f0} (D/flink-demo/.../SumWindowFunction.java:
 * 8-19), Beam's keep {@code KV.getKey()}; the shim rebuilds those objects from the GPU's number and the f0 / key of
 * the operator's tuples.  These combines keep {@code partialAggregate1}'s other fields, so the reference's result
 * carries the fields of the window's FIRST partial: the first tuple added to the first non-empty slice the window
 * contains (AggregateValueState.merge clones the first non-empty partial and folds the rest into it,
 * S/state/AggregateValueState.java:55-69).  A stand-alone operator registers the hidden SCOTTY_AGG_FIRST column,
 * gets that tuple's arrival index per window and rebuilds the fields from the tuple itself (the benchmark's
 * {@code SumAggregation} Tuple4 -- f0, f2, f3 of the first tuple, B/flinkBenchmark/aggregations/SumAggregation.java:
 * 16-18 -- and the demos' Tuple2 / KV under GlobalScottyWindowOperator, whose f0 varies).  A per-key operator of the
 * keyed engine has no FIRST column: there the rebuild uses the instance's one f0 / key -- exact for the keyed
 * connectors (one operator per key, F/KeyedScottyWindowOperator.java:56-62) -- and throws at the next
 * processWatermark if an instance sees two different ones; Tuple4 functions are refused there.
 */
public final class NativeFunctions {

    private NativeFunctions() {
    }

    /** How a registered function reads its tuples and rebuilds its result. */
    enum Shape {
        NUMBER,     // Integer / Long / Double tuples, boxed result
        TUPLE2_F1,  // org.apache.flink.api.java.tuple.Tuple2: value f1, result new Tuple2(f0, value)
        KV_VALUE,   // org.apache.beam.sdk.values.KV: value getValue(), result KV.of(getKey(), value)
        TUPLE4_F1,  // org.apache.flink.api.java.tuple.Tuple4: value f1, result new Tuple4(f0, value, f2, f3) of the
                    // window's first partial's tuple (B/flinkBenchmark/aggregations/SumAggregation.java:16-18)
    }

    enum Op { SUM, COUNT, MIN, MAX }

    static final class Spec {
        private final Op op;
        private final Shape shape;

        Spec(Op op, Shape shape) {
            this.op = op;
            this.shape = shape;
        }

        Op op() {
            return op;
        }

        Shape shape() {
            return shape;
        }
    }

    /** The reference's shipped functions with GPU semantics (file: lift / combine / lower restated). */
    static final Map<String, Spec> REGISTRY = new HashMap<>();

    static {
        String d = "de.tub.dima.scotty.demo.";
        // D/flink-demo/.../windowFunctions/{Sum,Min,Max}WindowFunction.java: Tuple2<Integer,Integer>, f1 combined
        REGISTRY.put(d + "flink.windowFunctions.SumWindowFunction", new Spec(Op.SUM, Shape.TUPLE2_F1));
        REGISTRY.put(d + "flink.windowFunctions.MinWindowFunction", new Spec(Op.MIN, Shape.TUPLE2_F1));
        REGISTRY.put(d + "flink.windowFunctions.MaxWindowFunction", new Spec(Op.MAX, Shape.TUPLE2_F1));
        // D/{kafka,samza,spark}-demo/.../windowFunctions/{Sum,Min,Max}WindowFunction.java: Integer
        for (String p : new String[]{"kafkaStreams", "samza", "spark"}) {
            REGISTRY.put(d + p + ".windowFunctions.SumWindowFunction", new Spec(Op.SUM, Shape.NUMBER));
            REGISTRY.put(d + p + ".windowFunctions.MinWindowFunction", new Spec(Op.MIN, Shape.NUMBER));
            REGISTRY.put(d + p + ".windowFunctions.MaxWindowFunction", new Spec(Op.MAX, Shape.NUMBER));
        }
        // D/storm-demo/.../windowFunctions/{Sum,Min,Max,Count}.java: Integer (Count: lift 1, combine +)
        REGISTRY.put(d + "storm.windowFunctions.Sum", new Spec(Op.SUM, Shape.NUMBER));
        REGISTRY.put(d + "storm.windowFunctions.Min", new Spec(Op.MIN, Shape.NUMBER));
        REGISTRY.put(d + "storm.windowFunctions.Max", new Spec(Op.MAX, Shape.NUMBER));
        REGISTRY.put(d + "storm.windowFunctions.Count", new Spec(Op.COUNT, Shape.NUMBER));
        // D/beam-demo/.../windowFunctions/{Sum,Min,Max,Count}.java: KV<Integer,Integer>, value combined, key kept
        REGISTRY.put(d + "beam.windowFunctions.Sum", new Spec(Op.SUM, Shape.KV_VALUE));
        REGISTRY.put(d + "beam.windowFunctions.Min", new Spec(Op.MIN, Shape.KV_VALUE));
        REGISTRY.put(d + "beam.windowFunctions.Max", new Spec(Op.MAX, Shape.KV_VALUE));
        REGISTRY.put(d + "beam.windowFunctions.Count", new Spec(Op.COUNT, Shape.KV_VALUE));
        // B/flinkBenchmark/aggregations/SumAggregation.java: Tuple4<String,Integer,Long,Long>, f1 summed, the first
        // partial's f0 / f2 / f3 kept (a stand-alone operator's SCOTTY_AGG_FIRST column)
        REGISTRY.put("de.tub.dima.scotty.flinkBenchmark.aggregations.SumAggregation", new Spec(Op.SUM, Shape.TUPLE4_F1));
    }

    /** Functions known by name whose result cannot be rebuilt: rejected with a reason (none at present). */
    static final Map<String, String> REJECTED = Collections.emptyMap();

    static int kindFor(Op op, int valueType) {
        switch (op) {
            case COUNT:
                return AGG_COUNT;
            case SUM:
                return valueType == VALUE_I32 ? AGG_SUM_I32 : valueType == VALUE_I64 ? AGG_SUM_I64 : AGG_SUM_F64;
            case MIN:
                return valueType == VALUE_I32 ? AGG_MIN_I32 : valueType == VALUE_I64 ? AGG_MIN_I64 : AGG_MIN_F64;
            default:
                return valueType == VALUE_I32 ? AGG_MAX_I32 : valueType == VALUE_I64 ? AGG_MAX_I64 : AGG_MAX_F64;
        }
    }

    /**
     * The binding of a function for an operator of the given value type, or an UnsupportedOperationException naming
     * why it has none.
     */
    @SuppressWarnings({"unchecked", "rawtypes"})
    static Binding bind(AggregateFunction<?, ?, ?> fn, int valueType) {
        final int inv = fn instanceof InvertibleAggregateFunction ? AGG_INVERTIBLE : 0;
        if (fn instanceof NativeValues.NativeKind) {
            NativeValues.NativeKind k = (NativeValues.NativeKind) fn;
            int kind = k.scottyKind();
            if (kind < 0 || (kind & 0xFFFF) > AGG_MAX_F64)
                throw new UnsupportedOperationException("NativeKind " + fn.getClass().getName() + " states kind " + kind);
            return new Binding(kind | inv, null, k);
        }
        String name = fn.getClass().getName();
        String why = REJECTED.get(name);
        if (why != null) throw new UnsupportedOperationException(why);
        Spec spec = REGISTRY.get(name);
        if (spec == null)
            throw new UnsupportedOperationException("AggregateFunction without a GPU kind (user lambdas and functions "
                    + "not in NativeFunctions.REGISTRY cannot run on the GPU; implement NativeValues.NativeKind): "
                    + name);
        return new Binding(kindFor(spec.op(), valueType) | inv, spec, null);
    }

    /**
     * One registered function of one operator instance: its kind, the value a tuple contributes, the result
     * rebuild, and the instance's exemplar tuple (f0 / key of its results).
     */
    static final class Binding {
        final int kind;  // SCOTTY_AGG_* | AGG_INVERTIBLE
        private final Spec spec;
        @SuppressWarnings("rawtypes")
        private final NativeValues.NativeKind user;
        private Object exemplar;
        private Object exemplarKey;
        private boolean keyVaries;
        private MethodHandle valueOf, keyOf, f2Of, f3Of;
        private Constructor<?> tuple2;
        private Method kvOf;

        @SuppressWarnings("rawtypes")
        Binding(int kind, Spec spec, NativeValues.NativeKind user) {
            this.kind = kind;
            this.spec = spec;
            this.user = user;
        }

        /** The result keeps fields of the window's first partial's tuple (the SCOTTY_AGG_FIRST column rebuilds it). */
        boolean keepsFirst() {
            return user == null && spec.shape() != Shape.NUMBER;
        }

        /** Only the first partial's tuple can rebuild the result (no per-instance exemplar suffices). */
        boolean needsFirst() {
            return user == null && spec.shape() == Shape.TUPLE4_F1;
        }

        /** A copy for another operator instance (same function, its own exemplar). */
        Binding fresh() {
            return new Binding(kind, spec, user);
        }

        /** The number the function's lift reads from {@code tuple} (COUNT: unused, the GPU lifts 1). */
        @SuppressWarnings("unchecked")
        Number value(Object tuple) {
            if (exemplar == null) exemplar = tuple;
            if (user != null) return user.scottyValue(tuple);
            switch (spec.shape()) {
                case NUMBER:
                    return spec.op() == Op.COUNT ? 1 : NativeValues.number(tuple);
                default: {
                    try {
                        if (valueOf == null) accessors(tuple.getClass());
                        Object k = keyOf.invoke(tuple);
                        if (exemplarKey == null && tuple == exemplar) exemplarKey = k;
                        else if (!Objects.equals(k, exemplarKey)) keyVaries = true;
                        return spec.op() == Op.COUNT ? 1 : (Number) valueOf.invoke(tuple);
                    } catch (Throwable t) {
                        throw new IllegalArgumentException("cannot read " + spec.shape() + " tuple " + tuple, t);
                    }
                }
            }
        }

        private void accessors(Class<?> cls) throws ReflectiveOperationException {
            MethodHandles.Lookup l = MethodHandles.publicLookup();
            if (spec.shape() == Shape.TUPLE2_F1 || spec.shape() == Shape.TUPLE4_F1) {
                valueOf = l.findGetter(cls, "f1", Object.class);
                keyOf = l.findGetter(cls, "f0", Object.class);
                if (spec.shape() == Shape.TUPLE4_F1) {
                    f2Of = l.findGetter(cls, "f2", Object.class);
                    f3Of = l.findGetter(cls, "f3", Object.class);
                }
            } else {
                valueOf = l.findVirtual(cls, "getValue", MethodType.methodType(Object.class));
                keyOf = l.findVirtual(cls, "getKey", MethodType.methodType(Object.class));
            }
        }

        /**
         * The reference's lower() result for one window's lowered word.  first: the window's first partial's tuple
         * (SCOTTY_AGG_FIRST; null on a per-key operator, which uses its one f0 / key).
         */
        @SuppressWarnings("unchecked")
        Object rebuild(long bits, Object first) {
            Object boxed = NativeValues.box(kind, bits);
            if (user != null) return user.scottyRebuild(boxed, exemplar);
            if (spec.shape() == Shape.NUMBER) return boxed;
            if (first == null && (keyVaries || spec.shape() == Shape.TUPLE4_F1))
                throw new UnsupportedOperationException("the tuples of one operator carry different "
                        + (spec.shape() == Shape.KV_VALUE ? "keys" : "fields") + ": the reference's result keeps the "
                        + "window's first partial's, which this operator has no SCOTTY_AGG_FIRST column for (a per-key "
                        + "operator of the keyed engine; use a stand-alone operator, or a NativeKind function)");
            try {
                Object src = first != null ? first : exemplar;
                if (valueOf == null) accessors(src.getClass());
                Object key = first != null ? keyOf.invoke(first) : exemplarKey;
                if (spec.shape() == Shape.TUPLE2_F1) {
                    if (tuple2 == null) tuple2 = src.getClass().getConstructor(Object.class, Object.class);
                    return tuple2.newInstance(key, boxed);
                }
                if (spec.shape() == Shape.TUPLE4_F1) {
                    if (tuple2 == null)
                        tuple2 = src.getClass().getConstructor(Object.class, Object.class, Object.class, Object.class);
                    return tuple2.newInstance(key, boxed, f2Of.invoke(first), f3Of.invoke(first));
                }
                if (kvOf == null) {
                    Class<?> kv = Class.forName("org.apache.beam.sdk.values.KV", true, src.getClass().getClassLoader());
                    kvOf = kv.getMethod("of", Object.class, Object.class);
                }
                return kvOf.invoke(null, key, boxed);
            } catch (RuntimeException e) {
                throw e;
            } catch (Throwable e) {
                throw new IllegalStateException("cannot rebuild " + spec.shape() + " result", e);
            }
        }
    }
}
