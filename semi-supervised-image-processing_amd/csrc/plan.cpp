// Launch plans (include/ssip.h "Launch plans"): a recorded sequence of the
// library's stream-ordered entry points, replayed from C++.
//
// Why: one eager train step is ~250 launches; enqueued from Python each costs
// ~25 us of interpreter + ctypes + allocator work (the step was within ~10 %
// of being host-bound).  A hipGraph removes that cost but HIP runs a graph's
// parallel branches one after another, which loses the weak-forward and
// side-stream wgrad overlap.  A plan keeps both: replay is a tight C++ loop
// over typed calls with fixed pointers, and cross-stream order is kept with
// the same event record / wait pairs the eager step uses.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <stdlib.h>

#include <memory>
#include <vector>

#include "../../include/ssip.h"
#include "stop_event.h"

namespace ssip {
void set_error(const char* fmt, ...);
}

namespace {

inline float plan_f32(uint64_t v) {
  uint32_t u = (uint32_t)v;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
inline double plan_f64(uint64_t v) {
  double d;
  memcpy(&d, &v, 8);
  return d;
}

struct PlanFn {
  const char* name;
  int nargs;
  int (*call)(const uint64_t* a);
};

#include "plan_thunks.inc"

constexpr int kNumFns = (int)(sizeof(kPlanFns) / sizeof(kPlanFns[0]));

enum OpKind { OP_CALL = 0, OP_EVENT = 1, OP_WAIT = 2, OP_MARK = 3 };

struct Op {
  int kind;
  int fn;          // OP_CALL
  int64_t arg0;    // OP_CALL: first slot in Plan::slots
  int event;       // OP_EVENT / OP_WAIT
  hipStream_t stream;
};

}  // namespace

struct ssip_plan {
  std::vector<Op> ops;
  std::vector<Op> ilv;               // ops re-ordered stream by stream (interleave_segments)
  std::vector<int> fuse;             // per ilv op: the event an OP_CALL records as its completion, or -1
  std::vector<int> nlaunch;          // per ilv op: launches the OP_CALL made on its stream (-1: not counted yet)
  size_t ilv_ops = (size_t)-1;       // ops.size() when ilv was built
  std::vector<uint64_t> slots;
  std::vector<std::unique_ptr<uint8_t[]>> blobs;
  std::vector<hipEvent_t> events;
  std::vector<size_t> seg_begin{0};  // op index where each segment starts
  ~ssip_plan() {
    for (hipEvent_t e : events) (void)hipEventDestroy(e);
  }
};

extern "C" {

ssip_plan* ssip_plan_create(void) { return new (std::nothrow) ssip_plan(); }

void ssip_plan_destroy(ssip_plan* plan) { delete plan; }

int ssip_plan_fn_index(const char* name) {
  if (!name) return -1;
  for (int i = 0; i < kNumFns; ++i)
    if (strcmp(kPlanFns[i].name, name) == 0) return i;
  return -1;
}

int ssip_plan_add_call(ssip_plan* plan, int fn, int nargs, const uint64_t* slots, const int64_t* blob_len,
                       const void* blob_data) {
  if (!plan || fn < 0 || fn >= kNumFns || nargs != kPlanFns[fn].nargs || (nargs && !slots)) {
    ::ssip::set_error("ssip_plan_add_call: bad plan, function index %d or argument count %d", fn, nargs);
    return SSIP_ERR_ARG;
  }
  Op op{OP_CALL, fn, (int64_t)plan->slots.size(), -1, nullptr};
  const uint8_t* bd = static_cast<const uint8_t*>(blob_data);
  for (int i = 0; i < nargs; ++i) {
    uint64_t v = slots[i];
    if (blob_len && blob_len[i] > 0) {
      if (!bd) {
        ::ssip::set_error("ssip_plan_add_call: blob argument %d without data", i);
        return SSIP_ERR_ARG;
      }
      std::unique_ptr<uint8_t[]> b(new (std::nothrow) uint8_t[blob_len[i]]);
      if (!b) {
        ::ssip::set_error("ssip_plan_add_call: out of host memory");
        return SSIP_ERR_ARG;
      }
      memcpy(b.get(), bd, (size_t)blob_len[i]);
      bd += blob_len[i];
      v = (uint64_t)(uintptr_t)b.get();
      plan->blobs.push_back(std::move(b));
    }
    plan->slots.push_back(v);
  }
  plan->ops.push_back(op);
  return SSIP_OK;
}

int ssip_plan_add_event(ssip_plan* plan, void* stream) {
  if (!plan) return SSIP_ERR_ARG;
  hipEvent_t e;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
    ::ssip::set_error("ssip_plan_add_event: hipEventCreateWithFlags failed");
    return SSIP_ERR_LAUNCH;
  }
  plan->events.push_back(e);
  const int id = (int)plan->events.size() - 1;
  plan->ops.push_back(Op{OP_EVENT, -1, 0, id, (hipStream_t)stream});
  return id;
}

int ssip_plan_add_wait(ssip_plan* plan, void* stream, int event) {
  if (!plan || event < 0 || event >= (int)plan->events.size()) {
    ::ssip::set_error("ssip_plan_add_wait: unknown event %d", event);
    return SSIP_ERR_ARG;
  }
  plan->ops.push_back(Op{OP_WAIT, -1, 0, event, (hipStream_t)stream});
  return SSIP_OK;
}

int ssip_plan_add_marker(ssip_plan* plan) {
  if (!plan) return SSIP_ERR_ARG;
  plan->seg_begin.push_back(plan->ops.size());
  return (int)plan->seg_begin.size() - 1;
}

int ssip_plan_segments(const ssip_plan* plan) { return plan ? (int)plan->seg_begin.size() : -1; }

int64_t ssip_plan_num_ops(const ssip_plan* plan) { return plan ? (int64_t)plan->ops.size() : -1; }

}  // extern "C"

namespace {

hipStream_t op_stream(const ssip_plan* plan, const Op& op) {
  if (op.kind == OP_CALL) return (hipStream_t)(uintptr_t)plan->slots[op.arg0 + kPlanFns[op.fn].nargs - 1];
  return op.stream;
}

// Enqueue order of a replay: the recorded order puts ALL of a segment's
// weak-forward launches (side stream) ahead of the train forward's (main
// stream), so the host spends the first ~60 launches feeding one stream while
// the other sits empty.  Within each segment, deal the ops out stream by
// stream, one per stream per turn, keeping each stream's own order; a wait is
// held back until the event it waits on has been recorded (issued) -- the
// device-side order the recording established is unchanged.
void interleave_segments(ssip_plan* plan) {
  plan->ilv.clear();
  plan->ilv.reserve(plan->ops.size());
  const size_t nseg = plan->seg_begin.size();
  std::vector<char> recorded(plan->events.size(), 0);
  for (size_t sg = 0; sg < nseg; ++sg) {
    const size_t b = plan->seg_begin[sg];
    const size_t e = sg + 1 < nseg ? plan->seg_begin[sg + 1] : plan->ops.size();
    std::vector<hipStream_t> streams;
    std::vector<std::vector<size_t>> q;
    for (size_t i = b; i < e; ++i) {
      const hipStream_t st = op_stream(plan, plan->ops[i]);
      size_t k = 0;
      while (k < streams.size() && streams[k] != st) ++k;
      if (k == streams.size()) {
        streams.push_back(st);
        q.emplace_back();
      }
      q[k].push_back(i);
    }
    std::vector<size_t> cur(streams.size(), 0);
    size_t left = e - b;
    while (left > 0) {
      bool progress = false;
      for (size_t k = 0; k < streams.size(); ++k) {
        // this stream's next op; events and waits do not count as a turn
        while (cur[k] < q[k].size()) {
          const Op& op = plan->ops[q[k][cur[k]]];
          if (op.kind == OP_WAIT && !recorded[op.event]) break;  // its record is not issued yet
          plan->ilv.push_back(op);
          if (op.kind == OP_EVENT) recorded[op.event] = 1;
          ++cur[k];
          --left;
          progress = true;
          if (op.kind == OP_CALL) break;
        }
      }
      if (!progress) {  // cannot happen for a recorded plan (every wait follows its record); keep the order
        plan->ilv.assign(plan->ops.begin(), plan->ops.end());
        plan->ilv_ops = plan->ops.size();
        return;
      }
    }
  }
  plan->ilv_ops = plan->ops.size();
  // an OP_CALL whose stream's next op is an event record records that event as
  // its launches' completion (SSIP_KLAUNCH); the record op itself is then skipped
  plan->fuse.assign(plan->ilv.size(), -1);
  plan->nlaunch.assign(plan->ilv.size(), -1);
  const bool off = getenv("SSIP_PLAN_MARKERS") != nullptr;  // A/B: separate marker packets
  for (size_t i = 0; i < plan->ilv.size() && !off; ++i) {
    const Op& op = plan->ilv[i];
    if (op.kind != OP_CALL) continue;
    const hipStream_t st = op_stream(plan, op);
    for (size_t j = i + 1; j < plan->ilv.size(); ++j) {
      const Op& nx = plan->ilv[j];
      if (nx.kind == OP_MARK || op_stream(plan, nx) != st) continue;
      if (nx.kind == OP_EVENT) plan->fuse[i] = (int)j;
      break;
    }
  }
}

}  // namespace

extern "C" {

int ssip_plan_run(ssip_plan* plan, int segment) {
  if (!plan || segment < 0 || segment >= (int)plan->seg_begin.size()) {
    ::ssip::set_error("ssip_plan_run: bad plan or segment %d", segment);
    return SSIP_ERR_ARG;
  }
  const size_t b = plan->seg_begin[segment];
  const size_t e = segment + 1 < (int)plan->seg_begin.size() ? plan->seg_begin[segment + 1] : plan->ops.size();
  if (plan->ilv_ops != plan->ops.size()) interleave_segments(plan);
  const std::vector<Op>& seq = plan->ilv;
  std::vector<char> done(e - b, 0);  // event records made by the launch before them
  for (size_t i = b; i < e; ++i) {
    const Op& op = seq[i];
    switch (op.kind) {
      case OP_CALL: {
        const int f = plan->fuse[i];
        ::ssip::StopEvent& se = ::ssip::stop_event();
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        const hipStream_t st = op_stream(plan, op);
        if (f >= 0 && (size_t)f < e && hipStreamIsCapturing(st, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone) {
          // first replay: count the op's launches on st; later: the last one records the event
          se.ev = plan->nlaunch[i] > 0 ? plan->events[seq[f].event] : nullptr;
          se.st = st;
          se.count = 0;
          se.target = plan->nlaunch[i] > 0 ? plan->nlaunch[i] : -1;
          se.used = 0;
        }
        const int rc = kPlanFns[op.fn].call(plan->slots.data() + op.arg0);
        const bool fused = se.ev != nullptr && se.used == 1 && se.count == se.target;
        if (se.st != nullptr && plan->nlaunch[i] < 0) plan->nlaunch[i] = se.count;
        se = ::ssip::StopEvent{};
        if (rc != SSIP_OK) return rc;  // the entry point set the message
        if (fused) done[f - b] = 1;  // else the record op below makes it
        break;
      }
      case OP_EVENT:
        if (done[i - b]) break;
        if (hipEventRecord(plan->events[op.event], op.stream) != hipSuccess) {
          ::ssip::set_error("ssip_plan_run: hipEventRecord failed at op %zu", i);
          return SSIP_ERR_LAUNCH;
        }
        break;
      case OP_WAIT:
        if (hipStreamWaitEvent(op.stream, plan->events[op.event], 0) != hipSuccess) {
          ::ssip::set_error("ssip_plan_run: hipStreamWaitEvent failed at op %zu", i);
          return SSIP_ERR_LAUNCH;
        }
        break;
      default:
        break;
    }
  }
  return SSIP_OK;
}

}  // extern "C"
