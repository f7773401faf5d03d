"""The reference's built-in incident catalogue (``test_all.py:40-50``), verbatim.

These are fixtures (data, not code): the ten k8s error messages the
reference's drivers analyse.  :func:`..synth.generate_cluster` with
``reference_incidents=True`` injects each one as an EVENT on an entity chain of
its fault type, so the reference's own driver scripts -- which hard-code these
messages -- find them in the synthetic stategraph (``tests/test_compat.py``).
"""

REFERENCE_INCIDENTS = [
    ('quota_pods',
     'Error creating: pods "es-white-list-cronjob-1607752440-gprx7" is forbidden: exceeded quota: compute-resources-dumeng1, requested: pods=1, used: pods=50, limited: pods=50'),
    ('nfs_missing',
     'MountVolume.SetUp failed for volume "pvc-f3788c43-6ca2-42fa-a1b5-7e760b6c4ff3" : mount failed: exit status 32 Mounting command: systemd-run Mounting arguments: --description=Kubernetes transient mount for /var/lib/kubelet/pods/92f33868-35c6-487f-8631-b2206363510a/volumes/kubernetes.io~nfs/pvc-f3788c43-6ca2-42fa-a1b5-7e760b6c4ff3 --scope -- mount -t nfs 172.16.112.63:/mnt/k8s_nfs_pv/chongni1-common-redis-pvc-0-common-redis-0-0-pvc-f3788c43-6ca2-42fa-a1b5-7e760b6c4ff3 /var/lib/kubelet/pods/92f33868-35c6-487f-8631-b2206363510a/volumes/kubernetes.io~nfs/pvc-f3788c43-6ca2-42fa-a1b5-7e760b6c4ff3 Output: Running scope as unit: run-re511f81c07574a6a84df041848b3347f.scope mount.nfs: mounting 172.16.112.63:/mnt/k8s_nfs_pv/chongni1-common-redis-pvc-0-common-redis-0-0-pvc-f3788c43-6ca2-42fa-a1b5-7e760b6c4ff3 failed, reason given by server: No such file or directory'),
    ('secret_missing',
     'MountVolume.SetUp failed for volume "es-account-token-k29vm" : secret "es-account-token-k29vm" not found'),
    ('configmap_missing',
     'MountVolume.SetUp failed for volume "gen-white-list-conf" : configmap "es-gen-white-list-configmap" not found'),
    ('cni_failure',
     'Failed create pod sandbox: rpc error: code = Unknown desc = failed to set up sandbox container "9a71227eb35345ead771b9f20ce90e2402641784c1866710c64adaaf0fbac1f2" network for pod "es-cronjob-1607813100-dqqg6": networkPlugin cni failed to set up pod "es-cronjob-1607813100-dqqg6_fanxy1" network: failed to Statfs "/proc/12631/ns/net": no such file or directory'),
    ('pvc_unbound',
     'pod has unbound immediate PersistentVolumeClaims'),
    ('nfs_stale',
     'MountVolume.SetUp failed for volume "pvc-6d127f0b-216d-4bb0-a967-6620c1671be6" : stat /var/lib/kubelet/pods/131523d6-21b1-4d85-bfef-da4fbde98991/volumes/kubernetes.io~nfs/pvc-6d127f0b-216d-4bb0-a967-6620c1671be6: stale NFS file handle'),
    ('pvc_deleting',
     'Unable to attach or mount volumes: unmounted volumes=[example-pv-storage], unattached volumes=[example-pv-storage default-token-l4rcp]: error processing PVC lizhiliang1/example-pvc1: PVC is being deleted'),
    ('sts_quota_memory',
     'create Pod yanghao71-c2-0 in StatefulSet yanghao71-c2 failed error: pods "yanghao71-c2-0" is forbidden: exceeded quota: compute-resources-yanghao71, requested: limits.memory=60Gi, used: limits.memory=1778Gi, limited: limits.memory=1800Gi'),
    ('sts_quota_pods',
     'create Pod yanghao71-c2-0 in StatefulSet yanghao71-c2 failed error: pods "yanghao71-c2-0" is forbidden: exceeded quota: compute-resources-yanghao71, requested: pods=1, used: pods=50, limited: pods=50'),
]
