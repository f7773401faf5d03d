"""``check_state/analyze_root_cause.py`` path (stage 3, A17-A23)."""
from k8s_llm_rca_amd.pipeline.check_state import (ad_hoc_find_entity_name, check_semantic, check_statepath,
                                                  check_states_existence_and_semantic, check_states_of_entity,
                                                  find_loose_states, find_strict_states,
                                                  setup_state_semantic_analyzer)

__all__ = ["setup_state_semantic_analyzer", "find_loose_states", "find_strict_states", "check_statepath",
           "check_states_of_entity", "ad_hoc_find_entity_name", "check_semantic",
           "check_states_existence_and_semantic"]
