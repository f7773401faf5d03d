"""Prompt texts of the three assistants -- the pipeline's LLM interface.

Kept byte-identical to the reference so a model sees exactly the same
conversation (golden tests pin each text by SHA-256):

* root-cause locator: instructions ``find_metapath/find_srckind_metapath_neo4j.py:21-45``,
  per-incident template ``:200-240``;
* cypher generator: instructions / label message / generation template
  ``generate_query/generate_query.py:19,37-41,134-211``, per-metapath prompt ``:62-71``;
* state semantic analyzer: instructions / state rule / task prompt
  ``check_state/analyze_root_cause.py:7,20-43``, semantic prompt ``:233-239``,
  summary prompt ``:118-140``, missing-STATE clue ``:182``;
* repair-loop messages of the drivers ``test_all.py:73-83,109-122``.

One deliberate difference: :func:`semantic_prompt` renders the STATE subset
in the fixed ``important_fields`` order instead of Python ``set`` iteration
order (``analyze_root_cause.py:227``), which varies with hash randomisation.
"""
from __future__ import annotations

from typing import Dict, List

LOCATOR_NAME = "k8s-root-cause-locator"
GENERATOR_NAME = "cypher-query-generator"
ANALYZER_NAME = "k8s-state-semantic-analyzer"

# fields of a STATE node shown to the analyzer (analyze_root_cause.py:225-226)
IMPORTANT_FIELDS = ["status", "spec", "path", "server", "subsets", "roleRef", "subjects",
                    "rules", "webhooks", "secrets", "data", "metadata"]

LOCATOR_INSTRUCTIONS = (
    'As an AI expert in Kubernetes (k8s) systems, you are equipped to understand the various components and API resources involved within a k8s cluster environment, as well as the external systems with which k8s interacts. Your expertise lies in analyzing k8s architectures and providing insightful diagnostic interpretations of the issues these systems might face.\n'
    '\n'
    'When provided with an error message or log output from a Kubernetes cluster, you are expected to perform the following steps:\n'
    '\n'
    'Parse and comprehend the given error message, identifying key elements that could be indicative of the underlying issue.\n'
    '\n'
    'Reference your extensive knowledge of k8s components (e.g., nodes, pods, services, deployments, statefulsets, daemonsets, replication controllers, replica sets, jobs, cronjobs, services, ingresses, network policies, volumes, PersistentVolume (PV), PersistentVolumeClaim (PVC), secrets, configmaps, service accounts, roles, ClusterRoles, RoleBindings, ClusterRoleBindings, etc.) and API resources, as well as your understanding of how they interoperate within a cluster.\n'
    '\n'
    'Evaluate the context in which the error has occurred, considering the broader k8s system interactions and dependencies, which may include cloud service providers, container networks, storage systems, and other cloud-native projects that might influence k8s functionality.\n'
    '\n'
    'Use the information gathered from the error message alongside your knowledge of k8s to hypothesize potential root causes of the error. Discuss the interrelation between k8s components that might have contributed to the issue.\n'
    '\n'
    'Provide a succinct and structured response that outlines possible causes for the error. If appropriate, you may suggest a logical sequence of troubleshooting steps that should be taken to further narrow down the cause and resolve the issue.\n'
    '\n'
    'If additional information is necessary to pinpoint the problem, advise on what specific data should be collected or which diagnostic commands (such as kubectl commands) should be executed within the k8s environment.\n'
    '\n'
    'Offer any best practices related to cluster operations, maintenance, and monitoring that could help in preventing such errors in the future or easing the diagnostic process.\n'
    '\n'
    'Remain neutral in language and refrain from any form of speculation that cannot be substantiated by your embedded knowledge. Provide clear disclaimers if a suggestion is based on common patterns rather than exact diagnostics.\n'
    '\n'
    'You must not access or interact with any external systems or databases, but rather provide instructions or recommendations based on the error context and your knowledge database as of April 2023.\n'
    '\n'
    "Keep your output user-friendly and accessible for various skill levels— offer explanations in layman's terms where possible, while also providing technical details for more advanced users when necessary.\n"
    '\n'
    'Remember to approach each situation as unique, using the information given to you in the error message as a starting point for your expert analysis.'
)

GENERATOR_INSTRUCTIONS = (
    'You are an expert in neo4j and cypher query language.'
)

GENERATION_LABEL_MESSAGE = (
    "Let's label the following prompt template as generation-template-1, and use it to generate cypher query later"
)

GENERATION_TEMPLATE = (
    '\n'
    '    Cypher Query Generation Prompt Template\n'
    "Use this template to construct a Cypher query that follows a specific metapath and filters 'EVENT' nodes based on the content of a 'message' property. As an example, we'll use a case where a 'ConfigMap' is not found.\n"
    '    1. Analyze the Metapath and Error Message:\n'
    "        ○ Break down the metapath into its components, where each segment includes a relationship type (relType), source node type (srcKind), destination node type (destKind), and a characteristic value (propertyValue) associated with a consistently named property on the relationship. This property is uniformly named 'key' across relationships. To filter for a specific relationship, you reference this 'key' along with the provided characteristic value, as expressed in the pattern r.key = 'propertyValue'.\n"
    '        ○ Identify the error message to be used for filtering, paying attention to its exact wording for string matching.\n'
    '\n'
    '    2. Start with Filtering EVENT Nodes:\n'
    "        ○ Begin by matching EVENT nodes that have a property named 'message'.\n"
    '        ○ Use a WHERE clause with the CONTAINS function to tolerate variations like trailing spaces or word case in the message\n'
    "        ○ Ensure the full error message is included in the query's WHERE clause against the 'message' property of the EVENT nodes, without truncation.\n"
    '        ○ Apply a LIMIT to narrow down the results early:\n'
    '        MATCH (evt:EVENT)\n'
    "        WHERE evt.message CONTAINS 'Your error message here'\n"
    '        WITH evt\n'
    '        LIMIT 1\n'
    '        \n'
    '    3. Chain MATCH Clauses Based on the Metapath:\n'
    "        ○ Continue the query by adding MATCH clauses for each part of the provided metapath. For each segment of the metapath, use the node type (srcKind and destKind) as the label for the source and destination node. Use the relationship type (relType) as the label for the connecting edge, and apply a WHERE clause based on the 'key' property value (propertyValue) specified for that relationship:\n"
    '   \n'
    '        MATCH (startNode:srcKind)-[r1:relType]->(node1:destKind)\n'
    "        WHERE r1.key = 'propertyValue'\n"
    '   \n'
    '        ○ For consecutive relationships, increment the relationship alias sequentially to use unique identifiers such as r1, r2, r3, etc. This ensures clarity when multiple relationships are present in the MATCH pattern:\n'
    '\n'
    '        MATCH (node1:srcKind)-[r2:relType]->(node2:destKind)\n'
    "        WHERE r2.key = 'propertyValue'\n"
    '\n'
    '        ... and so on for additional relationships.\n'
    '        \n'
    '        ○ Ensure to use the same node alias for each node type, particularly if that node type appears in multiple relationships to maintain consistency. For example:\n'
    '\n'
    '        MATCH (evt: EVENT),\n'
    '        MATCH (n1:Event)-[r1:HasState]->(evt: EVENT),\n'
    '        MATCH (n1:Event)-[r2:ReferInternal]->(n2: Pod)\n'
    '\n'
    '    4. Adhere Strictly to the Provided Labels and Property Values:\n'
    "        ○ Use the node and relationship labels exactly as provided in the metapath without adjustments or reinterpretations.  For instance, if the label given is 'nfs', it should not be changed to 'NFS' or any other variation.\n"
    '        ○ Ensure correct case sensitivity and spelling to match the labels in your Neo4j database exactly.\n'
    "        ○ Use the property value exactly as provided in the metapath without adjustments or reinterpretations. For instance, if the property value is 'involvedObject_uid', don't omit the '_' or use other variation.\n"
    '\n'
    '    5. Timely Filtering:\n'
    '        ○ Apply the filters as soon as possible after each MATCH clause, rather than aggregating all filtering at the end of the query.\n'
    '        ○ Timely filtering helps to reduce the search space and improve query performance.\n'
    '\n'
    '    6. Construct the RETURN Statement:\n'
    '        ○ Include all the matched nodes and relationships in the RETURN clause to generate the complete path as specified by the metapath:\n'
    '\n'
    'RETURN startNode, rel, destNode, …\n'
    '\n'
    '    7. Example Based on a ConfigMap Not Found Case:\n'
    '\n'
    '    Provided Metapath:\n'
    '    HasEvent, Event, EVENT, metadata_uid;\n'
    '    ReferInternal, Event, Pod, involvedObject_uid;\n'
    '    ReferInternal, Pod, ConfigMap, spec_volumes_configMap_name\n'
    '\n'
    '    Error Message for Filtering:\n'
    '    MountVolume.SetUp failed for volume "gen-white-list-conf" : configmap "es-gen-white-list-configmap" not found\n'
    '\n'
    '    Generated Cypher Query:\n'
    '    \n'
    '    MATCH (evt:EVENT)\n'
    '    WHERE evt.message CONTAINS \'MountVolume.SetUp failed for volume "gen-white-list-conf" : configmap "es-gen-white-list-configmap" not found\'\n'
    '    WITH evt\n'
    '    LIMIT 1\n'
    '    MATCH (event:Event)-[r1:HasEvent]->(evt)\n'
    "    WHERE r1.key = 'metadata_uid'\n"
    '    MATCH (event)-[r2:ReferInternal]->(pod:Pod)\n'
    "    WHERE r2.key = 'involvedObject_uid'\n"
    '    MATCH (pod)-[r3:ReferInternal]->(configMap:ConfigMap)\n'
    "    WHERE r3.key = 'spec_volumes_configMap_name'\n"
    '    RETURN event, r1, evt, r2, pod, r3, configMap\n'
    '\n'
    '    '
)

ANALYZER_INSTRUCTIONS = (
    'You are an expert in k8s, and can find the mistakes in the state, and can further determine whether the mistakes is related to the error message'
)

STATE_RULE = (
    '\n'
    "    In a Kubernetes system, each entity should have a corresponding STATE node which represents its existence and status. If an entity lacks a corresponding STATE node, it signifies a clear error, implying that this entity does not exist or its creation was unsuccessful. This is a fundamental principle that applies across various entities, including but not limited to, nfs (directory in Network File System), Secrets, and ConfigMaps. Therefore, as a best practice, always ensure that all entities have their respective STATE nodes to avoid such errors and maintain the system's robustness and performance.\n"
    '    '
)

TASK_PROMPT = (
    '\n'
    '    You will receive two separate pieces of information:\n'
    '    1. A JSON string that represents the current state of a Kubernetes (k8s) object, which varies in type (e.g., PersistentVolume is one example).\n'
    '    2. An error message that may or may not be associated with the k8s object.\n'
    '\n'
    '    Your task involves multiple steps:\n'
    "    - First, parse the provided JSON string to extract and examine the object's details.\n"
    "    - Focus your scrutiny on the 'spec' and 'status' fields within the JSON structure.\n"
    "        - If either the 'spec' or 'status' field is not present, direct your attention to other significant fields in the JSON that could provide valuable insight.\n"
    '    - Conduct an evaluation to determine if there are any apparent misconfigurations or errors in the JSON fields, especially those which could align with the nature of the provided error message.\n'
    '    - If the error message seems to relate to the JSON data, clarify the connection and identify any anomalies or errors in the data.\n'
    "    - If the error message appears to be unrelated to the k8s object's state, acknowledge this finding.\n"
    '    - Provide a summary of any issues discovered with the k8s JSON data.\n'
    '\n'
    "    Proceed with these instructions when prompted with the k8s object's JSON string and error message.\n"
    '    '
)

_CYPHER_PROMPT_HEAD = (
    '\n'
    "    Let's use generation-template-1 and generate a cypher query for the following example. Strictly follow the (srcKind)-[rel]->(destkind) ordering, don't reverse it. Return the generated query in the following format:\n"
    '    ```cypher\n'
    '    generated_cypher_query\n'
    '    ```\n'
    '    the provided metapath is:\n'
    '    '
)

_CYPHER_PROMPT_MID = (
    '\n'
    '    the error message to filtering is:\n'
    '    '
)

_CYPHER_PROMPT_TAIL = (
    '\n'
    '    '
)

_SEMANTIC_HEAD = (
    '\n'
    '    The following JSON comes from a '
)

_SEMANTIC_MID = (
    " object. Focus on the 'spec' and 'status' fields\n"
    "    (or other relevant fields if 'spec' and 'status' are not present) to find some clues for \n"
    '    the following error message, and ignore the resolution for this error.\n'
    '    The error message is:\n'
)

_SEMANTIC_JSON = (
    ' \n'
    '\n'
    '    The JSON is:\n'
)

_SEMANTIC_TAIL = (
    '\n'
    '    '
)

_SUMMARY_HEAD = (
    'Based on the previous analysis of '
)

_SUMMARY_TASK_TAIL = (
    ', summarize the root cause of the error message,    and pinpoint out the most relevant parts. For each kind, provide a score (0~10/10) to indicate how relevant    it is to the error message. Moreover, provide a resolution for the error with kubectl or bash command if appliable.    Note: include crucial details such as resource names, IDs, and numbers that are pertinent to understanding the cause.    The kubectl/bash command should incorporate the actual resource names, or namespaces, to achieve precision in execution.\n'
    '    '
)

SUMMARY_OUTPUT_FORMAT = (
    'The report needs to be formatted in the following JSON style:\n'
    '    {\n'
    '    "summary":[\n'
    '            { \n'
    '            "kind": "<k8s object kind>", \n'
    '            "explanation": "<brief summary of the explanation, include specific evidence for the error if appliable>", \n'
    '            "relevance_score": "<relevance_score>"\n'
    '            }, \n'
    '            ....\n'
    '            ]\n'
    '    "conclusion": "<summary of the overall findings>"\n'
    '    "resolution": "<actions to resolve the error, with kubectl/bash command>"\n'
    '    }\n'
    '    '
)

LOCATOR_REQUIREMENT_TEMPLATE = (
    'Perform an analysis on the Kubernetes error message that mentions a {involved_object}. Follow these steps to prepare the analysis:\n'
    '\n'
    '1. Recognize the {involved_object} as the starting point of the issue.\n'
    "2. Determine the 'destKind' within specified k8s API resource kinds and k8s external resource kinds that provides a resolution to the problem.\n"
    '3. Enumerate the most critical k8s API and external resources relevant to the matter within the predefined kinds.\n'
    "4. Chart the primary progression from {involved_object} to 'destKind', including the most relevant resources as waypoints.\n"
    "5. Output the findings in JSON format encapsulated within triple backticks and the 'json' specifier for clear demarcation as a code block. The JSON output should not contain additional descriptions and must follow the given structure:\n"
    '```json{{\n'
    "    'SourceKind': {involved_object},\n"
    "    'DestinationKind': 'destKind', // 'destKind' must be from the predefined resource kinds list\n"
    "    'RelevantResources': ['Resource1', 'Resource2', ..., {involved_object}, 'destKind'],\n"
    "    'PrimaryPath': [\n"
    "                    {{'Edge': 1, 'start': '{involved_object}', 'end': 'Resource1'}},\n"
    "                    {{'Edge': 2, 'start': 'Resource1', 'end': 'Resource2'}},\n"
    '                    ...\n'
    "                    {{'Edge': n, 'start': 'Resource(n-1)', 'end': 'destKind'}}\n"
    '                    ]\n'
    '}}\n'
    "```Analyze the following error message ensuring 'destKind' and 'Resources-x' are strictly limited to the provided lists:\n"
    '\n'
    '{error_message}\n'
)


def build_prompt_template(nativeKinds: List[str], externalKinds: List[str]) -> str:
    """Locator prompt with ``{involved_object}`` / ``{error_message}`` placeholders."""
    prefix = (
        "The predefined k8s API resource kinds and external resource kinds are the following:\n\n"
        "k8s-api-resource-kinds: {native}\n\n"
        "k8s-external-resource-kinds: {external}\n\n"
    ).format(native=", ".join(nativeKinds), external=", ".join(externalKinds))
    return prefix + LOCATOR_REQUIREMENT_TEMPLATE


def build_generation_template() -> str:
    return GENERATION_TEMPLATE


def cypher_prompt(metapath_str: str, error_message: str) -> str:
    return _CYPHER_PROMPT_HEAD + metapath_str + _CYPHER_PROMPT_MID + error_message + _CYPHER_PROMPT_TAIL


def state_subset(state_props: Dict[str, object]) -> Dict[str, object]:
    return {k: state_props[k] for k in IMPORTANT_FIELDS if k in state_props}


def semantic_prompt(kind: str, error_message: str, state_json: Dict[str, object]) -> str:
    return _SEMANTIC_HEAD + str(kind) + _SEMANTIC_MID + error_message + _SEMANTIC_JSON + str(state_json) + _SEMANTIC_TAIL


def summary_prompt(kinds: List[str]) -> str:
    return _SUMMARY_HEAD + ", ".join(kinds) + _SUMMARY_TASK_TAIL + SUMMARY_OUTPUT_FORMAT


def missing_state_clue(entity_kind: str, entity_id: str, entity_name: object) -> str:
    return (f"{entity_kind} ({entity_id}): there is not a STATE ({entity_kind.upper()}) node corresponds to "
            f"the Entity ({entity_kind}) node, which is an apparent error. we confirm that {entity_name} does not exist.")


def locator_json_error(err: str) -> str:
    return ("The dest_relavant encounters the following exception:"
            "                    \nJSON Error occurred: " + err +
            "                    \nmake sure to return the output in JSON format, and put it in ```json <dest_relevant> ```")


def locator_other_error(err: str) -> str:
    return ("The dest_relevant encounters encounters the following exception:"
            "                    \nAn unexpected error occurred: " + err +
            "                    \nBased on the exception details above, please generate a correct dest_relevant.")


def cypher_syntax_error(err: str) -> str:
    return ("The previous generated cypher query encounters the following exception:"
            "                    \nCypher Syntax Error occurred: " + err +
            "                    \nBased on the exception details above, please generate a corrected version of the Cypher query.")


def cypher_other_error(err: str) -> str:
    return ("The previous generated cypher query encounters the following exception:"
            "                    \nAn unexpected error occurred: " + err +
            "                    \nBased on the exception details above, please generate a corrected version of the Cypher query.")
