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
 * the operator's tuples.  That is exact when every tuple of one operator instance carries the same f0 / key -- the
 * keyed connectors' case (one operator per key, F/KeyedScottyWindowOperator.java:56-62) -- and the shim checks it
 * per tuple: if an instance sees two different f0 / keys it throws at the next processWatermark instead of
 * returning a value the reference would not.  The benchmark's {@code SumAggregation} (Tuple4 whose f2 / f3 are the
 * window's first tuple's timestamps) cannot be rebuilt from a number and is rejected.
 */
public final class NativeFunctions {

    private NativeFunctions() {
    }

    /** How a registered function reads its tuples and rebuilds its result. */
    enum Shape {
        NUMBER,     // Integer / Long / Double tuples, boxed result
        TUPLE2_F1,  // org.apache.flink.api.java.tuple.Tuple2: value f1, result new Tuple2(f0, value)
        KV_VALUE,   // org.apache.beam.sdk.values.KV: value getValue(), result KV.of(getKey(), value)
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
    }

    /** Functions known by name whose result cannot be rebuilt from the GPU's number: rejected with a reason. */
    static final Map<String, String> REJECTED = Collections.singletonMap(
            "de.tub.dima.scotty.flinkBenchmark.aggregations.SumAggregation",
            "SumAggregation keeps the first partial's f0 / f2 / f3 (B/flinkBenchmark/aggregations/SumAggregation.java:"
                    + "14-17): the window's first tuple, which the GPU does not track; implement NativeKind on a "
                    + "function whose lower() is the sum only");

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
        private MethodHandle valueOf, keyOf;
        private Constructor<?> tuple2;
        private Method kvOf;

        @SuppressWarnings("rawtypes")
        Binding(int kind, Spec spec, NativeValues.NativeKind user) {
            this.kind = kind;
            this.spec = spec;
            this.user = user;
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
            if (spec.shape() == Shape.TUPLE2_F1) {
                valueOf = l.findGetter(cls, "f1", Object.class);
                keyOf = l.findGetter(cls, "f0", Object.class);
            } else {
                valueOf = l.findVirtual(cls, "getValue", MethodType.methodType(Object.class));
                keyOf = l.findVirtual(cls, "getKey", MethodType.methodType(Object.class));
            }
        }

        /** The reference's lower() result for one window's lowered word. */
        @SuppressWarnings("unchecked")
        Object rebuild(long bits) {
            Object boxed = NativeValues.box(kind, bits);
            if (user != null) return user.scottyRebuild(boxed, exemplar);
            if (spec.shape() == Shape.NUMBER) return boxed;
            if (keyVaries)
                throw new UnsupportedOperationException("the tuples of one operator carry different "
                        + (spec.shape() == Shape.TUPLE2_F1 ? "f0" : "keys") + ": the reference's result keeps the "
                        + "window's first partial's, which the GPU does not track (use the keyed connector, or a "
                        + "NativeKind function)");
            try {
                if (spec.shape() == Shape.TUPLE2_F1) {
                    if (tuple2 == null) tuple2 = exemplar.getClass().getConstructor(Object.class, Object.class);
                    return tuple2.newInstance(exemplarKey, boxed);
                }
                if (kvOf == null) {
                    Class<?> kv = Class.forName("org.apache.beam.sdk.values.KV", true,
                            exemplar.getClass().getClassLoader());
                    kvOf = kv.getMethod("of", Object.class, Object.class);
                }
                return kvOf.invoke(null, exemplarKey, boxed);
            } catch (ReflectiveOperationException e) {
                throw new IllegalStateException("cannot rebuild " + spec.shape() + " result", e);
            }
        }
    }
}
