// exact_batch.h -- argument block of the batch-parallel exact path (exact_batch.hip), shared by the host engine
// (exact_engine.cpp) and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "exact_common.h"

namespace scotty {

struct XSnap;  // batch-start snapshot (exact_batch.hip)
struct XBCtl;  // control block of the event pass / apply segments (exact_batch.hip)

struct XBArgs {
  const int64_t* ts;
  const void* val;
  int64_t n;
  int64_t ntiles;
  const XCfg* cfg;
  XState* st;              // op 0
  XSlices sl;
  XSess ss;
  XSnap* snap;
  int64_t* reach;          // [XMAXCTX * sesscap] prefix max of (end + gap) over batch-start sessions
  long long* tmax;         // [ntiles] tile max
  long long* pcarry;       // [ntiles] exclusive prefix max carry
  int64_t* ns_cnt;         // [XMAXCTX][ntiles] new sessions per tile -> exclusive offsets
  int64_t* ns_tot;         // [XMAXCTX]
  int64_t* ns_start;       // [XMAXCTX][ns_cap]
  int64_t* ns_pb;          // [XMAXCTX][ns_cap]
  int64_t ns_cap;
  int64_t* ev_cnt;         // [ntiles] events per tile -> exclusive offsets
  long long* seg_tail;     // [ntiles] max ts after the tile's last event (or tile max)
  int32_t* seg_has;        // [ntiles] tile has an event
  long long* m_carry;      // [ntiles] max ts since the last event before the tile
  uint32_t* evbits;        // [n/32+1] event bitmap
  int64_t* ev_pos;         // [ev_cap]
  int64_t* ev_t;
  int64_t* ev_v;
  long long* ev_m;         // max ts strictly between the previous event and this one (JMIN if none)
  int64_t ev_cap;
  XBCtl* ctl;
  int64_t* ep_pos;         // [ep_cap] epoch entries: event position, tail after it
  int32_t* ep_tail;
  int64_t ep_cap;
  int32_t vt;
  int32_t cfg_nctx_host;   // session windows (host copy, decides which passes run)
  int64_t* sufmin;         // [sc] suffix minimum of tStart over [i, tail) (unsorted slice lists only)
  long long* tmin;         // [ntiles] tile min (sessions: the quiet-tile test of xb_classify_kernel)
  long long* dbg;          // debugging aid (SCOTTY_XB_PROF): clock stamps of the event pass, or null
  int32_t* tjump;          // [ntiles] (sessions) some item after the tile's first exceeds the tile's running max
                           // by more than the smallest gap: only then can a tuple other than the first open a session
};

hipError_t xb_classify_phase(XBArgs& a, int phase, hipStream_t st);
hipError_t xb_events(XBArgs& a, hipStream_t st);
hipError_t xb_apply(XBArgs& a, hipStream_t st);
int64_t xb_tile();
size_t xb_snap_bytes();
size_t xb_ctl_bytes();

}  // namespace scotty
