// Per-launch host switches of the HIP launchers (knobs.h): one table, written
// only by k8s_set_knob (k8s_llm_rca_amd/knobs.py pushes it on library load).
#include "common.h"
#include "knobs.h"

namespace k8s {
static int g_knobs[kKnobCount] = {1, 1, 6, 1, 0, 0, 0, 0};
int knob(int id) { return (id >= 0 && id < kKnobCount) ? g_knobs[id] : 0; }
}  // namespace k8s

K8S_API int k8s_set_knob(int id, int value) {
  if (id < 0 || id >= k8s::kKnobCount) return (int)hipErrorInvalidValue;
  k8s::g_knobs[id] = value;
  return 0;
}
K8S_API int k8s_get_knob(int id) { return k8s::knob(id); }
