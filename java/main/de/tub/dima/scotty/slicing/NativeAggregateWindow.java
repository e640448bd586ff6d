package de.tub.dima.scotty.slicing;

import de.tub.dima.scotty.core.AggregateWindow;
import de.tub.dima.scotty.core.windowType.WindowMeasure;

import java.util.List;

/**
 * One window result of the MI355X operator: the fields of the reference's AggregateWindowState
 * (slicing/src/main/java/de/tub/dima/scotty/slicing/state/AggregateWindowState.java) as returned by
 * scotty_process_watermark -- bounds, measure, hasValue and the lowered value of every aggregation in
 * registration order (empty when hasValue() is false, as AggregateWindowState.getAggValues returns).
 */
public final class NativeAggregateWindow implements AggregateWindow<Object> {

    private final WindowMeasure measure;
    private final long start, end;
    private final boolean hasValue;
    private final List<Object> values;

    public NativeAggregateWindow(WindowMeasure measure, long start, long end, boolean hasValue, List<Object> values) {
        this.measure = measure;
        this.start = start;
        this.end = end;
        this.hasValue = hasValue;
        this.values = values;
    }

    @Override
    public WindowMeasure getMeasure() {
        return measure;
    }

    @Override
    public long getStart() {
        return start;
    }

    @Override
    public long getEnd() {
        return end;
    }

    @Override
    public List<Object> getAggValues() {
        return values;
    }

    @Override
    public boolean hasValue() {
        return hasValue;
    }

    @Override
    public String toString() {
        return "Window{measure=" + measure + ", start=" + start + ", end=" + end + ", values=" + values + "}";
    }
}
