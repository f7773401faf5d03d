"""Reference import paths, for drop-in migration.

Code written against freiris/k8s-llm-rca imports its modules by package
path (``from common.openai_generic_assistant import OpenAIGenericAssistant``,
``from find_metapath.find_srckind_metapath_neo4j import *`` ...).  The same
paths exist under ``k8s_llm_rca_amd.compat``; put this directory on
``sys.path`` (:func:`install`) and the reference's driver scripts import this
framework unchanged:

=================================================  ==========================================
reference module                                   implementation
=================================================  ==========================================
``common/openai_generic_assistant.py``             :mod:`k8s_llm_rca_amd.api.assistant`
``common/neo4j_query_executor.py``                 :mod:`k8s_llm_rca_amd.api.graph`
``find_metapath/find_srckind_metapath_neo4j.py``   :mod:`k8s_llm_rca_amd.pipeline.find_metapath`
``generate_query/generate_query.py``               :mod:`k8s_llm_rca_amd.pipeline.generate_query`
``check_state/analyze_root_cause.py``              :mod:`k8s_llm_rca_amd.pipeline.check_state`
=================================================  ==========================================

Remote services become in-process ones: the assistant runs on the default
:class:`~k8s_llm_rca_amd.api.service.AssistantService` (set it with
``set_default_service``; e.g. an engine-backed service), and
``Neo4jQueryExecutor(uri, user, password)`` accepts ``mem://name`` graphs or
graph files instead of ``bolt://`` URIs (user/password are ignored).
"""
import os
import sys

COMPAT_DIR = os.path.dirname(os.path.abspath(__file__))


def install() -> None:
    """Make the reference's top-level package names importable."""
    if COMPAT_DIR not in sys.path:
        sys.path.insert(0, COMPAT_DIR)
