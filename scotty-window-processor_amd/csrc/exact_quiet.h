// exact_quiet.h -- one-pass ("quiet batch") path of the non-keyed exact engine, shared by exact_engine.cpp and
// exact_quiet.hip.
//
// A micro-batch of an operator with session windows (Eager slices, no count windows) is "quiet" when no tuple of it
// can change the SessionContexts' structure or open a flexible slice:
//   * no in-order tuple jumps the running max by a session gap or more (no new session, SessionWindow.java:80-83;
//     no flexible edge, S/StreamSlicer.java:118-130), and
//   * every out-of-order tuple lies inside the last session of every context (updateContext is then a no-op and
//     checkSliceEdges receives no modification, S/SliceManager.java:64-71; SessionWindow.java:46-79).
// For such a batch the operator behaves like the context-free grid path: every tuple ends in the last slice with
// tStart <= ts of the FINAL slice list (slices appended later start above the running max, S/SliceManager.java:
// 27-38), the fixed edges follow the closed-form rule of slicing_kernels.hip (commit_kernel), and the sessions' only
// change is the last one's end moving to the batch max (shiftEnd, SessionWindow.java:72-74).  The batch is therefore
// ingested ONCE with the grid path's ingest kernel into per-cell partials (cells = retained slices ++ grid cells above
// the pending edge), and a one-workgroup commit verifies the quiet conditions from the ingest's per-tile maxima and
// counters (the per-tile and per-edge scans of the batch spread over many workgroups, exact_quiet.hip) and either
// commits (edges, slices, state, sessions) or returns every cell to identity so the host runs
// the event-exact batch path (exact_batch.hip) on the same batch.  No state is written before the verdict (the start
// band's lowered view start travels in DevMeta.view_s0, not in the slice store).
//
// Start band (one session context, Eager slices): out-of-order tuples t with max(s - gap, reach) < t < s, where s is
// the last session's start and reach the latest end + gap of the sessions before it, move that start down one record
// low at a time in the reference: SessionWindow.java:56-66 shiftStart (getSession :86 returns the last session for them;
// no merge, since t > reach), and SliceManager.checkSliceEdges (S/SliceManager.java:89-125) moves the edge between the
// slice si ending at s (findSliceByEnd, searched from the end) and si + 1 to t when si is movable (Flexible(1)).  Every
// such tuple then lands in si + 1 (the last slice with tStart <= t), and every other tuple where it would have without
// the band (the moved edge only crosses tuples of the band).  So a batch whose out-of-order tuples reach into the
// band is still one pass: the prep kernel lets the cell view start at si + 1 with the band's lower end as its start
// (DevMeta.view_s0: the ingest and the cell index see it, the slice store does not), the ingest records per-tile
// minima, and the commit moves the edge and the session start to the batch minimum (and sets the store's order bits as
// checkSliceEdges' note_order would).  When no slice ends anywhere in [band lower end, s] (the session opened without
// a flexible edge), every shift's findSliceByEnd misses and is skipped: the band's tuples then land where the plain
// quiet view puts them and only the session start moves; the verdict then checks the batch minimum (not the lowest
// touched cell's start, which lies below the band) against the band's lower end.  C3's pause step: the stream resumes with a new session
// whose start settles over the next ~500 ms of tuples -- rounds of the event-exact path before, one quiet pass now.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_common.h"
#include "exact_common.h"

namespace scotty {

enum : int32_t {
  XQ_NONE = 0,
  XQ_COMMITTED = 1,   // the batch was quiet and is committed
  XQ_NOT_QUIET = 2,   // a tuple may change the session structure / open a flexible slice: event-exact path
  XQ_STATE = 3,       // operator state outside the quiet path (not started, unsorted list, open session context ...)
  XQ_GRID = 4,        // the pending edge is not in the device grid or the batch passes the grid horizon
  XQ_CAPACITY = 5,    // the new slices do not fit behind the tail
};

struct XQCtl {
  int32_t result;       // XQ_*
  int32_t rebuild;      // the grid horizon is running short: rebuild at the next synchronisation point
  int64_t n_emit;       // slices appended by the committed batch
  int64_t lo_bound;     // lowest ts an out-of-order tuple may have (inside the last session of every context)
  int64_t min_gap;      // smallest session gap
  int64_t p_start;      // maxEventTime at batch start
  int64_t c0;           // currentCount at batch start
  int64_t pending;      // nextEdgeTs at batch start
  int64_t h_end;        // grid horizon end
  int64_t batch_max;    // maxEventTime after the committed batch
  int64_t why;          // XQ_NOT_QUIET: 1 late / past the horizon, 2 below lo_bound, 4 tile start jump, 8 item jump, 16 range
  int64_t ncand;        // grid points <= batch_max (scan kernel -> edge and commit kernels)
  int64_t jump_tile;    // XQ_NOT_QUIET: first arrival tile holding a session-gap jump (JMAX: none located)
  int64_t jump_pos;     // the prep's refusal: arrival index (< 64) of the first session-gap jump, else -1
  int64_t band_si;      // start band (see below): the slice ending at the last session's start; -2: no slice ends in
                        // the band (only the start moves); -1: no band
  int64_t band_s;       // start band: the last session's start at batch start (slice band_si + 1 starts there)
  int64_t batch_min;    // start band: the batch's lowest timestamp (scan kernel)
};

struct XQArgs {
  const int64_t* ts;
  int64_t n;
  int64_t tile;
  const XCfg* cfg;
  XState* st;
  XSlices sl;
  XSess ss;
  const int64_t* grid;   // union edge grid of the context-free time windows (host-built, from a pending edge)
  int64_t gcount;        // valid grid entries
  DevMeta* meta;         // ingest / cell-index view of the operator (written by the prep kernel)
  unsigned long long* c_cnt;
  long long* c_tmax;
  unsigned long long* c_part[NPART];
  long long* tilemax;
  long long* tilemin;    // per-tile minima (the ingest's MODE bit 3)
  long long* pmax;       // scratch [NT_MAX]: prefix maxima of the tile maxima (arrival order)
  int32_t* rank;         // scratch [gcap]
  int32_t* flag;         // scratch [gcap]
  int64_t* eg;           // scratch [gcap]: emitted edges by rank
  int64_t* epos;         // scratch [gcap]: arrival index of the tuple that appends each emitted edge
  XQCtl* ctl;
  int64_t margin;        // grid horizon margin (ms past the stream front) below which a rebuild is requested
  long long* dbg;        // nullable: clock stamps of the commit's phases (SCOTTY_XQ_PROF, a debugging aid)
  int32_t band;          // the start band may be used (one session context, Eager slices, tilemin set)
};

hipError_t launch_xq_prep(const XQArgs& a, hipStream_t st);
// after the ingest: xq_scan_kernel (1 workgroup: prefix maxima, batch max, candidates), xq_edges_kernel (many
// workgroups: the gap checks of every tile and one arrival tile per candidate edge), xq_commit_kernel (1 workgroup)
hipError_t launch_xq_commit(const XQArgs& a, hipStream_t st);

}  // namespace scotty
