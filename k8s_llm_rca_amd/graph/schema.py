"""Kubernetes resource schema used by the metagraph and the stategraph generator.

The reference keeps this schema inside a Neo4j "metagraph" that is not part
of its repository; it is reconstructed here from what the reference code reads
(SURVEY.md §1.6):

* kind nodes carry ``kind`` and ``category`` (``NativeEntity`` /
  ``ExternalEntity``; ``find_metapath/find_srckind_metapath_neo4j.py:63-72``);
* relationships are ``ReferInternal`` / ``UseExternal`` / ``HasEvent`` with
  ``srcKind``, ``destKind`` and ``key`` = the flattened JSON field path of the
  referencing field (``generate_query/generate_query.py:51-57,188-190``,
  ``test_generate_query.py:26``, ``bkp_generate_query.py:228-234``);
* external kinds are ``nfs``, ``hostPath``, ``container`` and ``image``
  (``generate_query.py:116-121``).
"""
from __future__ import annotations

from typing import Dict, List, Tuple

NATIVE_KINDS: List[str] = [
    "ClusterRole", "ClusterRoleBinding", "ConfigMap", "CronJob", "DaemonSet", "Deployment",
    "Endpoints", "Event", "HorizontalPodAutoscaler", "Ingress", "Job", "LimitRange", "Namespace",
    "NetworkPolicy", "Node", "PersistentVolume", "PersistentVolumeClaim", "Pod",
    "PodDisruptionBudget", "ReplicaSet", "ResourceQuota", "Role", "RoleBinding", "Secret",
    "Service", "ServiceAccount", "StatefulSet", "StorageClass",
]
EXTERNAL_KINDS: List[str] = ["container", "hostPath", "image", "nfs"]

# which property of an external entity holds its "name" (generate_query.py:111-121)
EXTERNAL_NAME_KEY: Dict[str, str] = {
    "nfs": "path", "hostPath": "path", "container": "containerName", "image": "imageName",
}

# (relType, srcKind, destKind, key)
META_EDGES: List[Tuple[str, str, str, str]] = [
    ("HasEvent", "Event", "EVENT", "metadata_uid"),
    # Pod references
    ("ReferInternal", "Pod", "Node", "spec_nodeName"),
    ("ReferInternal", "Pod", "Namespace", "metadata_namespace"),
    ("ReferInternal", "Pod", "ConfigMap", "spec_volumes_configMap_name"),
    ("ReferInternal", "Pod", "ConfigMap", "spec_containers_envFrom_configMapRef_name"),
    ("ReferInternal", "Pod", "Secret", "spec_volumes_secret_secretName"),
    ("ReferInternal", "Pod", "Secret", "spec_imagePullSecrets_name"),
    ("ReferInternal", "Pod", "PersistentVolumeClaim", "spec_volumes_persistentVolumeClaim_claimName"),
    ("ReferInternal", "Pod", "ServiceAccount", "spec_serviceAccountName"),
    ("ReferInternal", "Pod", "ReplicaSet", "metadata_ownerReferences_uid"),
    ("ReferInternal", "Pod", "StatefulSet", "metadata_ownerReferences_uid"),
    ("ReferInternal", "Pod", "DaemonSet", "metadata_ownerReferences_uid"),
    ("ReferInternal", "Pod", "Job", "metadata_ownerReferences_uid"),
    ("UseExternal", "Pod", "container", "spec_containers_name"),
    ("UseExternal", "Pod", "image", "spec_containers_image"),
    ("UseExternal", "Pod", "hostPath", "spec_volumes_hostPath_path"),
    # storage
    ("ReferInternal", "PersistentVolumeClaim", "PersistentVolume", "spec_volumeName"),
    ("ReferInternal", "PersistentVolumeClaim", "StorageClass", "spec_storageClassName"),
    ("ReferInternal", "PersistentVolumeClaim", "Namespace", "metadata_namespace"),
    ("ReferInternal", "PersistentVolume", "PersistentVolumeClaim", "spec_claimRef_uid"),
    ("ReferInternal", "PersistentVolume", "StorageClass", "spec_storageClassName"),
    ("UseExternal", "PersistentVolume", "nfs", "spec_nfs_path"),
    ("UseExternal", "PersistentVolume", "hostPath", "spec_hostPath_path"),
    # workload controllers
    ("ReferInternal", "ReplicaSet", "Deployment", "metadata_ownerReferences_uid"),
    ("ReferInternal", "ReplicaSet", "Namespace", "metadata_namespace"),
    ("ReferInternal", "Deployment", "Namespace", "metadata_namespace"),
    ("ReferInternal", "StatefulSet", "Namespace", "metadata_namespace"),
    ("ReferInternal", "StatefulSet", "Service", "spec_serviceName"),
    ("ReferInternal", "DaemonSet", "Namespace", "metadata_namespace"),
    ("ReferInternal", "Job", "CronJob", "metadata_ownerReferences_uid"),
    ("ReferInternal", "Job", "Namespace", "metadata_namespace"),
    ("ReferInternal", "CronJob", "Namespace", "metadata_namespace"),
    ("ReferInternal", "HorizontalPodAutoscaler", "Deployment", "spec_scaleTargetRef_name"),
    ("ReferInternal", "PodDisruptionBudget", "Namespace", "metadata_namespace"),
    # config / identity
    ("ReferInternal", "ConfigMap", "Namespace", "metadata_namespace"),
    ("ReferInternal", "Secret", "Namespace", "metadata_namespace"),
    ("ReferInternal", "ServiceAccount", "Secret", "secrets_name"),
    ("ReferInternal", "ServiceAccount", "Namespace", "metadata_namespace"),
    ("ReferInternal", "RoleBinding", "Role", "roleRef_name"),
    ("ReferInternal", "RoleBinding", "ServiceAccount", "subjects_name"),
    ("ReferInternal", "RoleBinding", "Namespace", "metadata_namespace"),
    ("ReferInternal", "Role", "Namespace", "metadata_namespace"),
    ("ReferInternal", "ClusterRoleBinding", "ClusterRole", "roleRef_name"),
    ("ReferInternal", "ClusterRoleBinding", "ServiceAccount", "subjects_name"),
    # network
    ("ReferInternal", "Service", "Namespace", "metadata_namespace"),
    ("ReferInternal", "Endpoints", "Service", "metadata_name"),
    ("ReferInternal", "Endpoints", "Pod", "subsets_addresses_targetRef_uid"),
    ("ReferInternal", "Ingress", "Service", "spec_rules_http_paths_backend_serviceName"),
    ("ReferInternal", "Ingress", "Namespace", "metadata_namespace"),
    ("ReferInternal", "NetworkPolicy", "Namespace", "metadata_namespace"),
    # policy
    ("ReferInternal", "ResourceQuota", "Namespace", "metadata_namespace"),
    ("ReferInternal", "LimitRange", "Namespace", "metadata_namespace"),
]

# every native kind can be the involved object of an Event
EVENT_TARGETS: List[str] = [k for k in NATIVE_KINDS if k != "Event"]


def category_of(kind: str) -> str:
    if kind in EXTERNAL_KINDS:
        return "ExternalEntity"
    if kind == "EVENT":
        return "EventState"
    return "NativeEntity"


def build_metagraph():
    """Kind-level schema graph (the reference's metagraph database)."""
    from .store import PropertyGraph

    g = PropertyGraph("metagraph")
    ids: Dict[str, int] = {}
    for k in NATIVE_KINDS + EXTERNAL_KINDS + ["EVENT"]:
        cat = category_of(k)
        ids[k] = g.add_node(cat, {"kind": k, "category": cat})
    edges = list(META_EDGES)
    for k in EVENT_TARGETS:
        edges.append(("ReferInternal", "Event", k, "involvedObject_uid"))
    for t, s, d, key in edges:
        g.add_edge(ids[s], ids[d], t, {"srcKind": s, "destKind": d, "key": key})
    return g.finalize()
