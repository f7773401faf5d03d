"""Golden-format tests: prompt texts and string builders are byte-identical to the reference.

Hashes were computed from the reference's own builders (imported under stub
SDKs); expected strings for the metapath/fallback builders are SURVEY.md §2 A12 / §3.4.
"""
import hashlib

from k8s_llm_rca_amd.graph.model import Path
from k8s_llm_rca_amd.pipeline import prompts as P
from k8s_llm_rca_amd.pipeline.generate_query import extend_metapath_construct_string, human_generate_cypher_query

GOLDEN = {
    "LOCATOR_INSTRUCTIONS": "bb62c1ed5b398b160382fe14fa062a0974cfabac68ca0959162cfb2e00fbcde0",
    "GENERATOR_INSTRUCTIONS": "4738e0ad8c845b956a470e0a2d173fe524ceed44fa4b9441caaca2cdfc7d4f9a",
    "GENERATION_LABEL_MESSAGE": "993c353b1c760462c8e094c9c341667d001180dd6e1acc1383380eaaea1272c9",
    "GENERATION_TEMPLATE": "6a6119ec7a1d6b0e56d22f1bc8693a2fdd95c72cf6f595ca4f3a1d26c2188715",
    "ANALYZER_INSTRUCTIONS": "3cd8131b2ad57fe47ebbdc00094d07a53d390ea77daf50ef751b56e7b3d27959",
    "STATE_RULE": "9906f167988e4fa9ff0cc917f7cabf8d45e7507116ce20b0639d2a3a70fb6efc",
    "TASK_PROMPT": "f212b316f0edbbf3f6e97d5fe0ac355b1e0b780d3dc6f1bc01c001bdc6294ab0",
}


def h(s):
    return hashlib.sha256(s.encode()).hexdigest()


def test_prompt_constants():
    for name, digest in GOLDEN.items():
        assert h(getattr(P, name)) == digest, name


def test_prompt_builders():
    assert h(P.build_prompt_template(["Pod", "Secret"], ["nfs"])) == \
        "de49559296daf49fd5d3bfdba6f0547586bc1641032b12aa4287cd4070cc87a5"
    assert h(P.cypher_prompt("MP", "EM")) == "45ae05241ec63c8599d843614d2d940a64b73ba5b0a3061dccb9c851cd79b9cc"
    assert h(P.summary_prompt(["Pod", "Secret"])) == "7f799a928624ed77a0e41afe76101b8a150ff9837000c88ddee04e5a15c43f33"
    assert h(P.semantic_prompt("Pod", "EM", {"status": "T", "spec": "S"})) == \
        "9af2f529e10d3c902293545c2732f3979f1e0b879014be664e1fe090c36044a8"


def test_locator_template_formats():
    t = P.build_prompt_template(["Pod"], ["nfs"])
    s = t.format(error_message="boom", involved_object="Pod")
    assert "k8s-api-resource-kinds: Pod" in s and s.rstrip().endswith("boom")
    assert "'SourceKind': Pod," in s


def test_missing_state_clue():
    c = P.missing_state_clue("nfs", "abc", "/mnt/x")
    assert c == ("nfs (abc): there is not a STATE (NFS) node corresponds to the Entity (nfs) node, "
                 "which is an apparent error. we confirm that /mnt/x does not exist.")


class _G:
    def node_props(self, i):
        return [{"kind": "Pod"}, {"kind": "Secret"}][i]

    def edge_props(self, i):
        return {"srcKind": "Pod", "destKind": "Secret", "key": "spec_volumes_secret_secretName"}

    def edge_type_name(self, i):
        return "ReferInternal"


def test_extend_metapath_string():
    from k8s_llm_rca_amd.graph.model import Node, Relationship
    g = _G()
    p = Path([Node(g, 0), Node(g, 1)], [Relationship(g, 0)])
    assert extend_metapath_construct_string(p) == (
        "\n    HasEvent, Event, EVENT, metadata_uid;\n    ReferInternal, Event, Pod, involvedObject_uid;\n"
        "    ReferInternal, Pod, Secret, spec_volumes_secret_secretName;\n")


def test_human_cypher_golden():
    mp = ("\n    HasEvent, Event, EVENT, metadata_uid;\n    ReferInternal, Event, Pod, involvedObject_uid;\n"
          "    ReferInternal, Pod, Secret, spec_volumes_secret_secretName;\n")
    msg = 'MountVolume.SetUp failed for volume "es-account-token-k29vm" : secret "es-account-token-k29vm" not found'
    expected = (
        "MATCH (evt:EVENT)\n"
        "WHERE evt.message CONTAINS 'MountVolume.SetUp failed for volume \"es-account-token-k29vm\" : secret "
        "\"es-account-token-k29vm\" not found'\n"
        "WITH evt\nLIMIT 1\n\n"
        "MATCH (n1:Event)-[r1:HasEvent]->(evt:EVENT)\nWHERE r1.key = 'metadata_uid'\n\n"
        "MATCH (n1:Event)-[r2:ReferInternal]->(n2:Pod)\nWHERE r2.key = 'involvedObject_uid'\n\n"
        "MATCH (n2:Pod)-[r3:ReferInternal]->(n3:Secret)\nWHERE r3.key = 'spec_volumes_secret_secretName'\n\n"
        "RETURN evt, r1, n1, r2, n2, r3, n3")
    assert human_generate_cypher_query(mp, msg) == expected


def test_human_cypher_quote_escape_and_assert():
    q = human_generate_cypher_query("A, Event, EVENT, k;", "it's \"x\" failed")
    assert "CONTAINS 'it\\'s \"x\" failed'" in q
    import pytest
    with pytest.raises(AssertionError):
        human_generate_cypher_query("R, A, B, k1;R, A, B, k2;R, B, A, k3;", "m")
