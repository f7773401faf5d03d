// Host-side switches the launchers consult per launch (A/B-able in one
// process).  Set from Python (k8s_llm_rca_amd/knobs.py, the only place the
// environment is read) through k8s_set_knob; the slots match knobs.NATIVE.
#pragma once

namespace k8s {
enum Knob : int {
  kKnobGldsHand = 0,        // gemm_stream.hip: hand-issued LDS reads in glds_strip (1)
  kKnobDecodeReducePre = 1, // attention.hip: decode reduce prefetch form (1)
  kKnobPfW8 = 2,            // attention.hip: prefill kernel variant (6; 1 = the default, 0 = pg64)
  kKnobPfMerge16 = 3,       // attention.hip: 16-B merge for bf16 partials (1)
  kKnobArFenceAll = 4,      // allreduce.hip: system fence in every wave (0)
  kKnobDecodeKvNt = 5,      // attention.hip: non-temporal K/V loads in the decode stream (0)
  kKnobCount = 8
};
int knob(int id);
}  // namespace k8s
