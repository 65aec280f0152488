// Launch-plan replay (plan.cpp): when the next op of a stream after an entry
// point is an event record, the replay hands the event here and the entry
// point's LAST launch on that stream (SSIP_KLAUNCH, ssip_common.h; the first
// replay counts an op's launches) records it as its completion --
// hipExtLaunchKernel's stop event -- instead of a separate marker packet: each
// such record sat as a ~6.5 us bubble in front of the next kernel of the main
// stream in the round-5 step trace, and so does every launch made with a stop
// event, hence only the last.
#pragma once
#include <hip/hip_runtime.h>

namespace ssip {
struct StopEvent {
  hipEvent_t ev = nullptr;
  hipStream_t st = nullptr;  // null: no plan op is being replayed
  int count = 0;             // launches on st so far in this op
  int target = -1;           // the launch (1-based) that records ev; -1: count only
  int used = 0;              // launches that recorded ev
};
StopEvent& stop_event();  // this thread's (abi.cpp)
}  // namespace ssip
