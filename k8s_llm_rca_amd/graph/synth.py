"""Synthetic Kubernetes stategraph generator with fault injection (G9).

The reference diagnoses incidents against a Neo4j dump of a real cluster that
is not in its repository.  This module builds an
equivalent instance-level graph deterministically from a seed:

* entity nodes labelled by kind (``id``, ``kind2``, ``isNative``, ``isAtomic``,
  ``name2``; external kinds carry ``tag`` + ``path`` / ``containerName`` /
  ``imageName``);
* STATE nodes labelled ``UPPER(kind)`` holding JSON-string ``spec`` /
  ``status`` / ``metadata`` and linked by ``HasState {tmin, tmax}``
  (half-open validity, ``check_state/analyze_root_cause.py:64-79``);
* ``Event -[:HasEvent {key:'metadata_uid'}]-> EVENT {message, timestamp}`` and
  ``Event -[:ReferInternal {key:'involvedObject_uid'}]-> involved entity``
  (``find_srckind_metapath_neo4j.py:76-84``);
* typed reference edges between entities following :mod:`.schema`.

Incidents reproduce the reference's catalogue (``test_all.py:40-50``): quota
exhausted (pods / memory), NFS directory missing, stale NFS handle, Secret or
ConfigMap missing, CNI sandbox failure, unbound PVC, PVC being deleted.  Each
:class:`Incident` records its ground truth (source kind, root-cause kind and
the kinds on the primary path) so tests can check the pipeline's answer.
"""
from __future__ import annotations

import json
import uuid
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

from .schema import EXTERNAL_NAME_KEY
from .store import PropertyGraph, ms_to_ts, ts_to_ms

T0 = ts_to_ms("2020-12-10 00:00:00.000")
WINDOW_MS = 4 * 24 * 3600 * 1000
FOREVER = "9999-12-31 23:59:59.999"
NODES_PER_INCIDENT = 2.85  # measured mean over FAULT_TYPES (Event + EVENT + re-stated / dangling object)

FAULT_TYPES = [
    "quota_pods", "nfs_missing", "secret_missing", "configmap_missing", "cni_failure",
    "pvc_unbound", "nfs_stale", "pvc_deleting", "sts_quota_memory", "sts_quota_pods",
]

_WORDS = ["es", "white", "list", "gen", "redis", "common", "console", "gemini", "ds", "api", "web",
          "cache", "db", "kafka", "zk", "etl", "ml", "train", "serve", "auth", "log", "metric",
          "proxy", "gw", "search", "index", "feed", "job", "batch", "report"]
_USERS = ["dumeng", "chongni", "fanxy", "lizhiliang", "yanghao", "zhangxianqing", "xuw", "wangli",
          "chenyu", "liuqi", "sunmin", "zhaolei", "qianwei", "zhouyi", "wuhao", "zhengkai"]


@dataclass
class Incident:
    fault: str
    message: str
    timestamp: str
    src_kind: str
    dest_kind: str
    path_kinds: List[str]
    involved_id: str
    root_id: str


@dataclass
class SynthCluster:
    stategraph: PropertyGraph
    metagraph: PropertyGraph
    incidents: List[Incident] = field(default_factory=list)
    seed: int = 0

    @property
    def messages(self) -> List[str]:
        return [i.message for i in self.incidents]


class _Gen:
    def __init__(self, seed: int):
        self.rng = np.random.default_rng(seed)
        self.g = PropertyGraph("stategraph")
        self.uid_ids: Dict[str, int] = {}
        self.kind_of: Dict[int, str] = {}
        self.names_used: Dict[str, int] = {}
        self.state_edges: Dict[int, List[int]] = {}
        self.msg_override: Optional[str] = None  # reference-catalogue injection: the event text to use

    # ---------------------------------------------------------------- names
    def uid(self) -> str:
        return str(uuid.UUID(bytes=self.rng.bytes(16), version=4))

    def word(self) -> str:
        return _WORDS[int(self.rng.integers(len(_WORDS)))]

    def suffix(self, n=5) -> str:
        a = "bcdfghjklmnpqrstvwxz2456789"
        return "".join(a[int(i)] for i in self.rng.integers(0, len(a), n))

    def unique(self, base: str) -> str:
        c = self.names_used.get(base, 0)
        self.names_used[base] = c + 1
        return base if c == 0 else f"{base}-{c}"

    def ts(self, lo_ms: int, hi_ms: int) -> str:
        return ms_to_ts(int(self.rng.integers(lo_ms, hi_ms)))

    # ------------------------------------------------------------- entities
    def entity(self, kind: str, name: str, ns: Optional[str], created_ms: int,
               spec: Optional[dict] = None, status: Optional[dict] = None,
               with_state: bool = True, extra_meta: Optional[dict] = None) -> Tuple[int, str]:
        u = self.uid()
        props = {"id": u, "kind2": kind, "isNative": "true", "isAtomic": "false", "name2": name}
        if ns:
            props["namespace"] = ns
        nid = self.g.add_node(kind, props)
        self.uid_ids[u] = nid
        self.kind_of[nid] = kind
        if with_state:
            meta = {"name": name, "uid": u, "creationTimestamp": ms_to_ts(created_ms)}
            if ns:
                meta["namespace"] = ns
            if extra_meta:
                meta.update(extra_meta)
            self.state(nid, kind, u, created_ms, None, spec, status, meta)
        return nid, u

    def external(self, tag: str, value: str, created_ms: int, with_state: bool = True,
                 state_props: Optional[dict] = None) -> Tuple[int, str]:
        u = self.uid()
        props = {"id": u, "tag": tag, "isNative": "false", "isAtomic": "false",
                 EXTERNAL_NAME_KEY[tag]: value}
        nid = self.g.add_node(tag, props)
        self.uid_ids[u] = nid
        self.kind_of[nid] = tag
        if with_state:
            sp = {"kind": tag, "id": u}
            sp.update(state_props or {})
            s = self.g.add_node(tag.upper(), sp)
            e = self.g.add_edge(nid, s, "HasState", {"tmin": ms_to_ts(created_ms), "tmax": FOREVER})
            self.state_edges.setdefault(nid, []).append(e)
        return nid, u

    def state(self, nid: int, kind: str, u: str, t_from: int, t_to: Optional[int],
              spec, status, meta) -> int:
        sp = {"kind": kind, "id": u, "metadata": json.dumps(meta, sort_keys=True)}
        if spec is not None:
            sp["spec"] = json.dumps(spec, sort_keys=True)
        if status is not None:
            sp["status"] = json.dumps(status, sort_keys=True)
        s = self.g.add_node(kind.upper(), sp)
        e = self.g.add_edge(nid, s, "HasState", {"tmin": ms_to_ts(t_from),
                                                 "tmax": FOREVER if t_to is None else ms_to_ts(t_to)})
        self.state_edges.setdefault(nid, []).append(e)
        return s

    def ref(self, a: int, b: int, key: str, rel: str = "ReferInternal") -> int:
        return self.g.add_edge(a, b, rel, {"key": key, "srcKind": self.kind_of[a], "destKind": self.kind_of[b]})

    def event(self, involved: int, message: str, ts: str, reason: str, etype: str = "Warning") -> int:
        if self.msg_override is not None and etype == "Warning":
            message = self.msg_override
        name = f"{self.g.node_props(involved).get('name2', 'obj')}.{self.suffix(16)}"
        ev, _ = self.entity("Event", name, self.g.node_props(involved).get("namespace"),
                            ts_to_ms(ts), with_state=False)
        st = self.g.add_node("EVENT", {"kind": "Event", "message": message, "timestamp": ts,
                                       "reason": reason, "type": etype,
                                       "id": self.g.node_props(ev)["id"]})
        self.g.add_edge(ev, st, "HasEvent", {"key": "metadata_uid"})
        self.ref(ev, involved, "involvedObject_uid")
        return ev


def generate_cluster(target_nodes: int = 10_000, n_incidents: int = 64, seed: int = 0,
                     fault_mix: Optional[List[str]] = None, reference_incidents: bool = False) -> SynthCluster:
    """Build a stategraph of ``target_nodes`` nodes (+- half a tenant, faults included) with
    ``n_incidents`` faults; at most ~30 % of the target is spent on fault nodes, beyond that the
    graph grows past the target (callers cycle a smaller incident set instead)."""
    from .schema import build_metagraph

    G = _Gen(seed)
    g = G.g
    rng = G.rng
    faults = list(fault_mix or FAULT_TYPES)

    # cluster-scoped objects
    n_nodes = max(2, target_nodes // 400)
    k8s_nodes = []
    for i in range(n_nodes):
        nid, _ = G.entity("Node", f"node-{i:03d}", None, T0 - WINDOW_MS,
                          spec={"podCIDR": f"10.{i // 250}.{i % 250}.0/24"},
                          status={"conditions": [{"type": "Ready", "status": "True"},
                                                 {"type": "NetworkUnavailable", "status": "False"}],
                                  "capacity": {"cpu": "96", "memory": "768Gi", "pods": "110"}})
        k8s_nodes.append(nid)
    sc, _ = G.entity("StorageClass", "nfs-client", None, T0 - WINDOW_MS,
                     spec={"provisioner": "cluster.local/nfs-client-provisioner"})
    nfs_server = "172.16.112.63"

    # per-namespace tenants.  Every injected incident adds ~2.85 nodes (its Event
    # entity + EVENT, plus a re-stated or dangling object), so the base is built
    # to the target minus that reserve, the faults are injected, and tenants are
    # added again until the final count lands on the target (+- half a tenant).
    reserve = min(int(target_nodes * 0.3), int(NODES_PER_INCIDENT * n_incidents))
    n0 = g.num_nodes
    tenants = [_add_tenant(G, k8s_nodes, sc, nfs_server)]
    while g.num_nodes + (g.num_nodes - n0) / len(tenants) < target_nodes - reserve:  # undershoot; topped up below
        tenants.append(_add_tenant(G, k8s_nodes, sc, nfs_server))
    tenant_size = (g.num_nodes - n0) / len(tenants)
    app_size = max(1.0, (tenant_size - 8) / 4.0)  # a tenant = ~8 fixed nodes + 2..6 apps

    # ------------------------------------------------------------ incidents
    incidents: List[Incident] = []
    tries = miss = 0
    while len(incidents) < n_incidents and tries < n_incidents * 20:
        tries += 1
        # the scheduled type (uniform mix) on up to 5 random tenants, then the next
        # type: a graph with no tenant able to host one fault type still fills up
        fault = faults[(len(incidents) + miss // 5) % len(faults)]
        t = tenants[int(rng.integers(len(tenants)))]
        inc = _inject(G, t, fault, nfs_server)
        if inc is None:
            miss += 1
        else:
            incidents.append(inc)
            miss = 0
    if reference_incidents:  # the reference's ten built-in messages, verbatim (reference_incidents.py)
        from .reference_incidents import REFERENCE_INCIDENTS
        for fault, message in REFERENCE_INCIDENTS:
            for _ in range(50):
                G.msg_override = message
                try:
                    inc = _inject(G, tenants[int(rng.integers(len(tenants)))], fault, nfs_server)
                finally:
                    G.msg_override = None
                if inc is not None:
                    inc.message = message
                    incidents.append(inc)
                    break
    while g.num_nodes + 8 + app_size / 2 < target_nodes:  # top up with tenants sized to the remainder
        n_apps = int(min(6, max(1, round((target_nodes - g.num_nodes - 8) / app_size))))
        _add_tenant(G, k8s_nodes, sc, nfs_server, n_apps)
    return SynthCluster(stategraph=g.finalize(), metagraph=build_metagraph(), incidents=incidents, seed=seed)


def _add_tenant(G: _Gen, k8s_nodes: List[int], sc: int, nfs_server: str, n_apps: Optional[int] = None) -> dict:
    """One namespace: quota, service-account token, 2-6 apps (deploy / sts / cron) with their pods."""
    g, rng = G.g, G.rng
    user = f"{_USERS[int(rng.integers(len(_USERS)))]}{int(rng.integers(1, 99))}"
    ns_name = G.unique(user)
    t_ns = T0 - WINDOW_MS + int(rng.integers(0, WINDOW_MS // 2))
    ns, _ = G.entity("Namespace", ns_name, None, t_ns, status={"phase": "Active"})
    quota_name = f"compute-resources-{ns_name}"
    quota, _ = G.entity("ResourceQuota", quota_name, ns_name, t_ns,
                        spec={"hard": {"pods": "50", "limits.memory": "1800Gi"}},
                        status={"hard": {"pods": "50", "limits.memory": "1800Gi"},
                                "used": {"pods": str(int(rng.integers(5, 40))),
                                         "limits.memory": f"{int(rng.integers(100, 900))}Gi"}})
    G.ref(quota, ns, "metadata_namespace")
    tok = f"default-token-{G.suffix(5)}"
    sa_secret, _ = G.entity("Secret", tok, ns_name, t_ns, spec=None,
                            status=None, extra_meta={"type": "kubernetes.io/service-account-token"})
    G.ref(sa_secret, ns, "metadata_namespace")
    sa, _ = G.entity("ServiceAccount", "default", ns_name, t_ns)
    G.ref(sa, ns, "metadata_namespace")
    G.ref(sa, sa_secret, "secrets_name")
    tenant = {"ns": ns, "ns_name": ns_name, "quota": quota, "quota_name": quota_name, "sa": sa,
              "sa_secret": sa_secret, "tok": tok, "pods": [], "jobs": [], "sts": [], "pvc_pods": []}
    n_draw = int(rng.integers(2, 7))
    for _ in range(n_apps or n_draw):
        kind = rng.choice(["deploy", "deploy", "sts", "cron"])
        app = G.unique(f"{G.word()}-{G.word()}-{ns_name}" if rng.random() < 0.3 else f"{G.word()}-{G.word()}")
        t_app = t_ns + int(rng.integers(0, WINDOW_MS // 4))
        cm, _ = G.entity("ConfigMap", f"{app}-configmap", ns_name, t_app,
                         extra_meta={"labels": {"app": app}})
        G.ref(cm, ns, "metadata_namespace")
        sec, _ = G.entity("Secret", f"{app}-secret", ns_name, t_app)
        G.ref(sec, ns, "metadata_namespace")
        svc, _ = G.entity("Service", app, ns_name, t_app, spec={"ports": [{"port": 8080}], "selector": {"app": app}})
        G.ref(svc, ns, "metadata_namespace")
        ep, _ = G.entity("Endpoints", app, ns_name, t_app)
        G.ref(ep, svc, "metadata_name")
        image_v = f"registry.local/{app}:v{int(rng.integers(1, 9))}.{int(rng.integers(0, 20))}"
        img, _ = G.external("image", image_v, t_app, state_props={"imageName": image_v})
        if kind == "deploy":
            dep, _ = G.entity("Deployment", app, ns_name, t_app, spec={"replicas": 2})
            G.ref(dep, ns, "metadata_namespace")
            rs_name = f"{app}-{G.suffix(10)}"
            owner, _ = G.entity("ReplicaSet", rs_name, ns_name, t_app, spec={"replicas": 2})
            G.ref(owner, dep, "metadata_ownerReferences_uid")
            G.ref(owner, ns, "metadata_namespace")
            pod_names = [f"{rs_name}-{G.suffix(5)}" for _ in range(2)]
        elif kind == "sts":
            owner, _ = G.entity("StatefulSet", app, ns_name, t_app, spec={"replicas": 2, "serviceName": app})
            G.ref(owner, ns, "metadata_namespace")
            G.ref(owner, svc, "spec_serviceName")
            tenant["sts"].append((owner, app))
            pod_names = [f"{app}-{i}" for i in range(2)]
        else:
            cj, _ = G.entity("CronJob", f"{app}-cronjob", ns_name, t_app, spec={"schedule": "*/5 * * * *"})
            G.ref(cj, ns, "metadata_namespace")
            stamp = 1607600000 + int(rng.integers(0, 300000))
            owner, _ = G.entity("Job", f"{app}-cronjob-{stamp}", ns_name, t_app, spec={"completions": 1})
            G.ref(owner, cj, "metadata_ownerReferences_uid")
            G.ref(owner, ns, "metadata_namespace")
            tenant["jobs"].append((owner, f"{app}-cronjob-{stamp}"))
            pod_names = [f"{app}-cronjob-{stamp}-{G.suffix(5)}"]
        for pn in pod_names:
            node = k8s_nodes[int(rng.integers(len(k8s_nodes)))]
            vol_cfg = f"{app}-conf"
            spec = {"nodeName": g.node_props(node)["name2"], "serviceAccountName": "default",
                    "containers": [{"name": app, "image": image_v}],
                    "volumes": [{"name": vol_cfg, "configMap": {"name": f"{app}-configmap"}},
                                {"name": f"{app}-secret", "secret": {"secretName": f"{app}-secret"}},
                                {"name": tok, "secret": {"secretName": tok}}]}
            pvc = pv = nfs = None
            if kind == "sts":
                pvc_name = f"pvc-{app}-{pn}"
                pvc, pvc_uid = G.entity("PersistentVolumeClaim", pvc_name, ns_name, t_app,
                                        spec={"storageClassName": "nfs-client"},
                                        status={"phase": "Bound"})
                pv_name = f"pvc-{pvc_uid}"
                path = f"/mnt/k8s_nfs_pv/{ns_name}-{pvc_name}-{pv_name}"
                pv, _ = G.entity("PersistentVolume", pv_name, None, t_app,
                                 spec={"nfs": {"server": nfs_server, "path": path},
                                       "claimRef": {"uid": pvc_uid, "name": pvc_name}},
                                 status={"phase": "Bound"})
                nfs, _ = G.external("nfs", path, t_app, state_props={"path": path, "server": nfs_server})
                G.ref(pvc, pv, "spec_volumeName")
                G.ref(pvc, sc, "spec_storageClassName")
                G.ref(pvc, ns, "metadata_namespace")
                G.ref(pv, pvc, "spec_claimRef_uid")
                G.ref(pv, sc, "spec_storageClassName")
                G.ref(pv, nfs, "spec_nfs_path", rel="UseExternal")
                spec["volumes"].append({"name": pv_name, "persistentVolumeClaim": {"claimName": pvc_name}})
            pod, pod_uid = G.entity("Pod", pn, ns_name, t_app + 1000, spec=spec,
                                    status={"phase": "Running", "hostIP": "172.16.0.1"})
            G.ref(pod, node, "spec_nodeName")
            G.ref(pod, ns, "metadata_namespace")
            G.ref(pod, cm, "spec_volumes_configMap_name")
            G.ref(pod, sec, "spec_volumes_secret_secretName")
            G.ref(pod, sa_secret, "spec_volumes_secret_secretName")
            G.ref(pod, sa, "spec_serviceAccountName")
            G.ref(pod, owner, "metadata_ownerReferences_uid")
            if pvc is not None:
                G.ref(pod, pvc, "spec_volumes_persistentVolumeClaim_claimName")
            ctr, _ = G.external("container", app, t_app + 1000, state_props={"containerName": app})
            G.ref(pod, ctr, "spec_containers_name", rel="UseExternal")
            G.ref(pod, img, "spec_containers_image", rel="UseExternal")
            G.ref(ep, pod, "subsets_addresses_targetRef_uid")
            rec = {"pod": pod, "pod_uid": pod_uid, "name": pn, "node": node, "cm": cm, "sec": sec,
                   "pvc": pvc, "pv": pv, "nfs": nfs, "app": app, "owner": owner}
            tenant["pods"].append(rec)
            if pvc is not None:
                tenant["pvc_pods"].append(rec)
            # a normal lifecycle event per pod
            G.event(pod, f"Successfully assigned {ns_name}/{pn} to {g.node_props(node)['name2']}",
                    G.ts(t_app + 1000, t_app + 5000), "Scheduled", "Normal")
    return tenant


def _pick(G: _Gen, items):
    return items[int(G.rng.integers(len(items)))] if items else None


def _inject(G: _Gen, t: dict, fault: str, nfs_server: str) -> Optional[Incident]:
    g = G.g
    ts_ms = T0 + int(G.rng.integers(WINDOW_MS // 2, WINDOW_MS))
    ts = ms_to_ts(ts_ms)
    ns_name = t["ns_name"]
    props = g.node_props

    if fault in ("quota_pods",):
        job = _pick(G, t["jobs"])
        if job is None:
            return None
        owner, jname = job
        pod = f"{jname}-{G.suffix(5)}"
        msg = (f'Error creating: pods "{pod}" is forbidden: exceeded quota: {t["quota_name"]}, '
               f"requested: pods=1, used: pods=50, limited: pods=50")
        _exhaust_quota(G, t, ts_ms, pods=True)
        G.event(owner, msg, ts, "FailedCreate")
        return Incident(fault, msg, ts, "Job", "ResourceQuota", ["Job", "Namespace", "ResourceQuota"],
                        props(owner)["id"], props(t["quota"])["id"])
    if fault in ("sts_quota_memory", "sts_quota_pods"):
        sts = _pick(G, t["sts"])
        if sts is None:
            return None
        owner, sname = sts
        if fault == "sts_quota_memory":
            req = "requested: limits.memory=60Gi, used: limits.memory=1778Gi, limited: limits.memory=1800Gi"
        else:
            req = "requested: pods=1, used: pods=50, limited: pods=50"
        msg = (f"create Pod {sname}-0 in StatefulSet {sname} failed error: pods \"{sname}-0\" is forbidden: "
               f"exceeded quota: {t['quota_name']}, {req}")
        _exhaust_quota(G, t, ts_ms, pods=(fault == "sts_quota_pods"))
        G.event(owner, msg, ts, "FailedCreate")
        return Incident(fault, msg, ts, "StatefulSet", "ResourceQuota",
                        ["StatefulSet", "Namespace", "ResourceQuota"], props(owner)["id"], props(t["quota"])["id"])
    if fault in ("nfs_missing", "nfs_stale", "pvc_unbound", "pvc_deleting"):
        rec = _pick(G, t["pvc_pods"])
        if rec is None:
            return None
        pod, pvc, pv, nfs = rec["pod"], rec["pvc"], rec["pv"], rec["nfs"]
        pv_name = props(pv)["name2"]
        pod_uid = rec["pod_uid"]
        mnt = f"/var/lib/kubelet/pods/{pod_uid}/volumes/kubernetes.io~nfs/{pv_name}"
        path = props(nfs)["path"]
        if fault == "nfs_missing":
            unit = f"run-r{G.suffix(32)}.scope"
            msg = (f'MountVolume.SetUp failed for volume "{pv_name}" : mount failed: exit status 32 Mounting command: '
                   f"systemd-run Mounting arguments: --description=Kubernetes transient mount for {mnt} --scope -- "
                   f"mount -t nfs {nfs_server}:{path} {mnt} Output: Running scope as unit: {unit} mount.nfs: mounting "
                   f"{nfs_server}:{path} failed, reason given by server: No such file or directory")
            _end_states(G, nfs, ts_ms - int(G.rng.integers(60_000, 3_600_000)))
            G.event(pod, msg, ts, "FailedMount")
            return Incident(fault, msg, ts, "Pod", "nfs",
                            ["Pod", "PersistentVolumeClaim", "PersistentVolume", "nfs"], rec["pod_uid"], props(nfs)["id"])
        if fault == "nfs_stale":
            msg = f'MountVolume.SetUp failed for volume "{pv_name}" : stat {mnt}: stale NFS file handle'
            _restate(G, nfs, "nfs", ts_ms - 120_000, None, {"path": path, "server": nfs_server,
                                                           "status": json.dumps({"exported": False, "fsid": "changed"})})
            G.event(pod, msg, ts, "FailedMount")
            return Incident(fault, msg, ts, "Pod", "nfs",
                            ["Pod", "PersistentVolumeClaim", "PersistentVolume", "nfs"], rec["pod_uid"], props(nfs)["id"])
        if fault == "pvc_unbound":
            msg = "pod has unbound immediate PersistentVolumeClaims"
            _restate_entity(G, pvc, ts_ms - 300_000, spec={"storageClassName": "nfs-client"},
                            status={"phase": "Pending"})
            G.event(pod, msg, ts, "FailedScheduling")
            return Incident(fault, msg, ts, "Pod", "PersistentVolumeClaim", ["Pod", "PersistentVolumeClaim"],
                            rec["pod_uid"], props(pvc)["id"])
        msg = (f"Unable to attach or mount volumes: unmounted volumes=[{pv_name}], unattached volumes=[{pv_name} "
               f"{t['tok']}]: error processing PVC {ns_name}/{props(pvc)['name2']}: PVC is being deleted")
        _restate_entity(G, pvc, ts_ms - 300_000, spec={"storageClassName": "nfs-client"},
                        status={"phase": "Bound"}, meta_extra={"deletionTimestamp": ms_to_ts(ts_ms - 300_000),
                                                              "finalizers": ["kubernetes.io/pvc-protection"]})
        G.event(pod, msg, ts, "FailedMount")
        return Incident(fault, msg, ts, "Pod", "PersistentVolumeClaim", ["Pod", "PersistentVolumeClaim"],
                        rec["pod_uid"], props(pvc)["id"])
    rec = _pick(G, t["pods"])
    if rec is None:
        return None
    pod = rec["pod"]
    if fault == "secret_missing":
        vol = f"{rec['app']}-token-{G.suffix(5)}"
        sec, _ = G.entity("Secret", vol, ns_name, ts_ms, with_state=False)  # referenced, never created
        G.ref(sec, t["ns"], "metadata_namespace")
        G.ref(pod, sec, "spec_volumes_secret_secretName")
        msg = f'MountVolume.SetUp failed for volume "{vol}" : secret "{vol}" not found'
        G.event(pod, msg, ts, "FailedMount")
        return Incident(fault, msg, ts, "Pod", "Secret", ["Pod", "Secret"], rec["pod_uid"], props(sec)["id"])
    if fault == "configmap_missing":
        vol = f"{rec['app']}-{G.suffix(4)}-conf"
        cm_name = f"{rec['app']}-{G.suffix(4)}-configmap"
        cm, _ = G.entity("ConfigMap", cm_name, ns_name, ts_ms, with_state=False)
        G.ref(cm, t["ns"], "metadata_namespace")
        G.ref(pod, cm, "spec_volumes_configMap_name")
        msg = f'MountVolume.SetUp failed for volume "{vol}" : configmap "{cm_name}" not found'
        G.event(pod, msg, ts, "FailedMount")
        return Incident(fault, msg, ts, "Pod", "ConfigMap", ["Pod", "ConfigMap"], rec["pod_uid"], props(cm)["id"])
    if fault == "cni_failure":
        node = rec["node"]
        sandbox = G.rng.bytes(32).hex()
        msg = (f'Failed create pod sandbox: rpc error: code = Unknown desc = failed to set up sandbox container '
               f'"{sandbox}" network for pod "{rec["name"]}": networkPlugin cni failed to set up pod '
               f'"{rec["name"]}_{ns_name}" network: failed to Statfs "/proc/{int(G.rng.integers(1000, 60000))}/ns/net": '
               f"no such file or directory")
        _restate_entity(G, node, ts_ms - 600_000, spec={"podCIDR": "10.0.0.0/24"},
                        status={"conditions": [{"type": "Ready", "status": "True"},
                                               {"type": "NetworkUnavailable", "status": "True",
                                                "reason": "CalicoIsDown"}]})
        G.event(pod, msg, ts, "FailedCreatePodSandBox")
        return Incident(fault, msg, ts, "Pod", "Node", ["Pod", "Node"], rec["pod_uid"], props(node)["id"])
    return None


def _end_states(G: _Gen, nid: int, end_ms: int) -> None:
    """Close every open STATE interval of ``nid`` at ``end_ms`` (entity disappears)."""
    g = G.g
    for e in G.state_edges.get(nid, []):
        p = g._e_props[e]
        if p.get("tmax") == FOREVER:
            if ts_to_ms(p["tmin"]) >= end_ms:
                p["tmin"] = ms_to_ts(end_ms - 1000)
            p["tmax"] = ms_to_ts(end_ms)


def _restate(G: _Gen, nid: int, kind: str, from_ms: int, spec, extra_props: dict) -> None:
    _end_states(G, nid, from_ms)
    g = G.g
    sp = {"kind": kind, "id": g.node_props(nid)["id"]}
    sp.update(extra_props)
    s = g.add_node(kind.upper(), sp)
    e = g.add_edge(nid, s, "HasState", {"tmin": ms_to_ts(from_ms), "tmax": FOREVER})
    G.state_edges.setdefault(nid, []).append(e)


def _restate_entity(G: _Gen, nid: int, from_ms: int, spec=None, status=None, meta_extra=None) -> None:
    g = G.g
    p = g.node_props(nid)
    kind = p["kind2"]
    _end_states(G, nid, from_ms)
    meta = {"name": p["name2"], "uid": p["id"]}
    if p.get("namespace"):
        meta["namespace"] = p["namespace"]
    if meta_extra:
        meta.update(meta_extra)
    G.state(nid, kind, p["id"], from_ms, None, spec, status, meta)


def _exhaust_quota(G: _Gen, t: dict, ts_ms: int, pods: bool) -> None:
    used = {"pods": "50", "limits.memory": "1000Gi"} if pods else {"pods": "31", "limits.memory": "1778Gi"}
    _restate_entity(G, t["quota"], ts_ms - 900_000, spec={"hard": {"pods": "50", "limits.memory": "1800Gi"}},
                    status={"hard": {"pods": "50", "limits.memory": "1800Gi"}, "used": used})
