"""``generate_query/generate_query.py`` path (stage 2, A11-A16)."""
from k8s_llm_rca_amd.pipeline.generate_query import (build_generation_template, extend_metapath_construct_string,
                                                     extract_cypher, generate_cypher_query,
                                                     human_generate_cypher_query, message_compatible,
                                                     run_and_filter_query, setup_cypher_generator)

__all__ = ["setup_cypher_generator", "extend_metapath_construct_string", "generate_cypher_query", "extract_cypher",
           "run_and_filter_query", "message_compatible", "build_generation_template", "human_generate_cypher_query"]
