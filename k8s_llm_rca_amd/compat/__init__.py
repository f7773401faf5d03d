"""Reference import paths, for drop-in migration.

Code written against freiris/k8s-llm-rca imports its modules by package
path (``from common.openai_generic_assistant import OpenAIGenericAssistant``,
``from find_metapath.find_srckind_metapath_neo4j import *`` ...).
:func:`install` puts an import hook first on ``sys.meta_path`` that serves
those paths from the table below (no files: each reference module is built
from this framework's implementation at import), so the reference's driver
scripts import this framework unchanged:

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
import importlib
import importlib.abc
import importlib.machinery
import os
import sys

COMPAT_DIR = os.path.dirname(os.path.abspath(__file__))
SHIMS_DIR = os.path.join(COMPAT_DIR, "shims")

_P = "k8s_llm_rca_amd."
# reference module -> (docstring, [(implementation module, names)], {class name: base class (module, name)})
# The two adapter classes keep their reference names as subclasses defined in the
# reference module (``openai_generic_assistant.py:11-14``, ``neo4j_query_executor.py:6-24``).
REFERENCE_MODULES = {
    "common.openai_generic_assistant": (
        "OpenAIGenericAssistant: no API key, no OpenAI() client; runs execute on the in-process service.",
        [], {"OpenAIGenericAssistant": (_P + "api.assistant", "GenericAssistant")}),
    "common.neo4j_query_executor": (
        "Neo4jQueryExecutor(uri, user, password) over an in-process graph (uri: mem://name or a graph file).",
        [(_P + "api.graph", ["register_graph"])], {"Neo4jQueryExecutor": (_P + "api.graph", "GraphQueryExecutor")}),
    "find_metapath.find_srckind_metapath_neo4j": (
        "Stage 1 (A3-A10): source kind, destination / relevant kinds, metapaths.",
        [(_P + "pipeline.find_metapath", ["setup_root_cause_locator", "find_native_external_kinds", "find_srcKind",
                                          "find_metapath", "print_metapath", "find_destKind_relevantResources",
                                          "extract_json"]),
         (_P + "pipeline.prompts", ["build_prompt_template"])], {}),
    "generate_query.generate_query": (
        "Stage 2 (A11-A16): metapath -> Cypher generation, execution and filtering.",
        [(_P + "pipeline.generate_query", ["setup_cypher_generator", "extend_metapath_construct_string",
                                           "generate_cypher_query", "extract_cypher", "run_and_filter_query",
                                           "message_compatible", "build_generation_template",
                                           "human_generate_cypher_query"])], {}),
    "check_state.analyze_root_cause": (
        "Stage 3 (A17-A23): state checks along a state path and the root-cause report.",
        [(_P + "pipeline.check_state", ["setup_state_semantic_analyzer", "find_loose_states", "find_strict_states",
                                        "check_statepath", "check_states_of_entity", "ad_hoc_find_entity_name",
                                        "check_semantic", "check_states_existence_and_semantic"])], {}),
}
REFERENCE_PACKAGES = sorted({m.split(".")[0] for m in REFERENCE_MODULES})


class _ReferencePaths(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    """Import hook serving :data:`REFERENCE_MODULES` (and their packages)."""

    def find_spec(self, name, path=None, target=None):
        if name in REFERENCE_MODULES or name in REFERENCE_PACKAGES:
            return importlib.machinery.ModuleSpec(name, self, is_package=name in REFERENCE_PACKAGES)
        return None

    def create_module(self, spec):
        return None

    def exec_module(self, mod):
        entry = REFERENCE_MODULES.get(mod.__name__)
        if entry is None:  # a package: its submodules come from this hook too
            mod.__doc__ = f"reference package path ``{mod.__name__}/`` (k8s_llm_rca_amd.compat)"
            return
        doc, names, classes = entry
        mod.__doc__ = doc
        exported = []
        for src, ns in names:
            impl = importlib.import_module(src)
            for n in ns:
                setattr(mod, n, getattr(impl, n))
            exported += ns
        for cname, (src, base) in classes.items():
            b = getattr(importlib.import_module(src), base)
            setattr(mod, cname, type(cname, (b,), {"__module__": mod.__name__, "__doc__": doc}))
            exported.append(cname)
        mod.__all__ = exported


_HOOK = _ReferencePaths()


def install(shims: bool = False) -> None:
    """Make the reference's top-level package names importable (the import
    hook, first on ``sys.meta_path``).  While the hook is installed it serves
    ``common.*``, ``find_metapath.*``, ``generate_query.*`` and ``check_state.*``
    with this framework's implementations, AHEAD of any reference checkout on
    ``sys.path``.  ``shims``: also put this framework's ``openai`` and ``neo4j``
    modules first on the path (``compat/shims``), so code that imports those
    SDKs runs on the in-process services; to run the reference's OWN adapter
    modules (``common/openai_generic_assistant.py`` /
    ``neo4j_query_executor.py``) over the shims, call :func:`uninstall` first
    so the checkout's files are imported (``tests/test_compat.py`` does).  Off
    by default: the shims shadow real installs of those packages."""
    if _HOOK not in sys.meta_path:
        sys.meta_path.insert(0, _HOOK)
    if shims and SHIMS_DIR not in sys.path:
        sys.path.insert(0, SHIMS_DIR)
        for mod in [m for m in sys.modules if m in ("openai", "neo4j") or m.startswith(("openai.", "neo4j."))]:
            del sys.modules[mod]


def uninstall() -> bool:
    """Remove the import hook and the reference-path modules it created (so a
    real checkout of the reference on ``sys.path`` is imported instead).
    Returns whether it was installed."""
    was = _HOOK in sys.meta_path
    if was:
        sys.meta_path.remove(_HOOK)
    for m in [m for m in sys.modules if m.split(".")[0] in REFERENCE_PACKAGES
              and getattr(sys.modules[m], "__loader__", None) is _HOOK]:
        del sys.modules[m]
    return was


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

