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

``install(shims=True)`` additionally provides ``openai`` (``OpenAI().beta.*``)
and ``neo4j`` (``GraphDatabase``, ``neo4j.graph``, ``neo4j.exceptions``)
modules backed by the same services, so the reference's own adapter and
driver modules import and run unmodified (``tests/test_compat.py``).

Remote services become in-process ones: the assistant runs on the default
:class:`~k8s_llm_rca_amd.api.service.AssistantService` (set it with
``set_default_service``; e.g. an engine-backed service), and
``Neo4jQueryExecutor(uri, user, password)`` accepts ``mem://name`` graphs or
graph files instead of ``bolt://`` URIs (user/password are ignored).
"""
import os
import sys

COMPAT_DIR = os.path.dirname(os.path.abspath(__file__))
SHIMS_DIR = os.path.join(COMPAT_DIR, "shims")


def install(shims: bool = False) -> None:
    """Make the reference's top-level package names importable.  ``shims``:
    also put this framework's ``openai`` and ``neo4j`` modules first on the
    path (``compat/shims``), so the reference's OWN adapter modules
    (``common/openai_generic_assistant.py`` / ``neo4j_query_executor.py``,
    which import those SDKs) run unchanged on the in-process services.  Off by
    default: it shadows real installs of those packages."""
    if COMPAT_DIR not in sys.path:
        sys.path.insert(0, COMPAT_DIR)
    if shims and SHIMS_DIR not in sys.path:
        sys.path.insert(0, SHIMS_DIR)
        for mod in [m for m in sys.modules if m in ("openai", "neo4j") or m.startswith(("openai.", "neo4j."))]:
            del sys.modules[mod]


def start_local(model: str = "llama3-8b", weights: str = None, tokenizer: str = None, device: str = None,
                graphs: dict = None, kv_gb: float = None, shims: bool = True):
    """One call for migrating drivers: start the in-process LLM engine on this
    GPU (``weights``: an HF checkpoint dir; random init otherwise), make it the
    default assistant service the ``openai`` shim talks to, register
    ``graphs`` (``{"bolt://host:7687": graph or graph-file path, ...}`` -- the
    URIs the driver hard-codes) for the ``neo4j`` shim, and :func:`install` the
    reference's import paths.  Returns the engine (``engine.stop()`` when done).
    """
    import torch

    from ..api.service import AssistantService, set_default_service
    from ..engine.backend import EngineBackend
    from ..engine.engine import EngineConfig, LLMEngine

    install(shims=shims)
    dev = device or ("cuda" if torch.cuda.is_available() else "cpu")
    cfg = EngineConfig(model=model, device=dev, dtype=torch.bfloat16 if dev != "cpu" else torch.float32,
                       kv_max_gb=kv_gb, num_blocks=None if dev != "cpu" else 1024, weights=weights,
                       tokenizer=tokenizer)
    eng = LLMEngine(cfg)
    eng.start()
    set_default_service(AssistantService(EngineBackend(eng)))
    if graphs:
        if not shims:
            raise ValueError("graphs= binds bolt:// URIs in the neo4j shim: needs shims=True")
        import neo4j  # the shim module install() put first on sys.path (the one driver code imports)
        for uri, g in graphs.items():
            neo4j.map_uri(uri, g)
    return eng

