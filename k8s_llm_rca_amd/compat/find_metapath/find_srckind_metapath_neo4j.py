"""``find_metapath/find_srckind_metapath_neo4j.py`` path (stage 1, A3-A10)."""
from k8s_llm_rca_amd.pipeline.find_metapath import (extract_json, find_destKind_relevantResources, find_metapath,
                                                    find_native_external_kinds, find_srcKind, print_metapath,
                                                    setup_root_cause_locator)
from k8s_llm_rca_amd.pipeline.prompts import build_prompt_template

__all__ = ["setup_root_cause_locator", "find_native_external_kinds", "find_srcKind", "find_metapath",
           "print_metapath", "find_destKind_relevantResources", "extract_json", "build_prompt_template"]
