"""Single schema source for the two pool kinds of group ``compute.my.domain/v1alpha1``.

Everything that describes the API surface is derived from the dicts in this file:

* ``config/crd/*.yaml`` (``make manifests`` -> ``scripts/gen_manifests.py``),
* the apiserver-sim's OpenAPI validation / defaulting / pruning (it loads the CRDs),
* ``native/include/gpupool/generated/schema_consts.h`` (group/version/plural/finalizer/
  condition-type constants used by the C++ controller), so Python and C++ cannot drift.

``AzureVmPool`` is wire-compatible with the reference guide's Go types
(``/root/reference/README.md:92-151``): same field names and json tags, ``replicas`` with
``+kubebuilder:validation:Minimum=0`` (README.md:94), a status subresource (README.md:131) and the
Desired/Ready printer columns (README.md:132-133). Fields without ``omitempty`` in the reference
are ``required`` here, exactly what controller-gen would emit.

``Mi355xPool`` is the MI355X-native kind: the same declarative
``spec.replicas``/``status.readyReplicas``/``conditions`` surface, reconciled against physical
gfx950 devices on an on-prem node instead of Azure VMs.
"""
from __future__ import annotations

import copy

GROUP = "compute.my.domain"
VERSION = "v1alpha1"
API_VERSION = f"{GROUP}/{VERSION}"

# Finalizer that guards device/VM release (reference roadmap README.md:309).
FINALIZER = "compute.my.domain/device-release"

# Well-known annotation/label keys shared by agent, manager and kubelet-fake.
ANN_AGENT_ENDPOINT = "gpupool.amd.com/agent-endpoint"
# the agent's X25519 key-exchange public key (base64url): the manager derives the per-node MAC
# key of its RPCs from it (gpupool/utils/edsig.py, v2)
ANN_AGENT_KX = "gpupool.amd.com/agent-kx"
ANN_POD_DEVICES = "gpupool.amd.com/devices"
LABEL_GFX = "amd.com/gpu.family"
LABEL_POOL = "gpupool.amd.com/pool"
DEFAULT_RESOURCE = "amd.com/gpu"

# Mi355xJob: finalizer that deletes the job's pods before the job goes away, and the labels every
# job pod carries (the controller lists pods by them and checks the owner UID).
JOB_FINALIZER = "compute.my.domain/job-cleanup"
LABEL_JOB = "gpupool.amd.com/job-name"
LABEL_JOB_INDEX = "gpupool.amd.com/replica-index"
LABEL_JOB_ATTEMPT = "gpupool.amd.com/attempt"
# Set on a running Mi355xJob by a higher-priority job that needs its GPUs ("<ns>/<name>/<uid>");
# the victim's own reconciler then stops its gang (single status writer per job).
ANN_JOB_PREEMPTED_BY = "gpupool.amd.com/preempted-by"
# Written by the pool autoscaler: time of its last spec.replicas change and the demand it saw.
ANN_AUTOSCALE_LAST = "gpupool.amd.com/autoscale-last-scale"
ANN_AUTOSCALE_DEMAND = "gpupool.amd.com/autoscale-demand"

# Condition types (metav1.Condition, README.md:126-127; roadmap README.md:310).
COND_READY = "Ready"
COND_PROGRESSING = "Progressing"
COND_DEGRADED = "Degraded"
COND_DELETING = "Deleting"
COND_CREDENTIALS = "CredentialsValid"
COND_XGMI = "XGMILinksHealthy"
COND_ECC = "HBMECCHealthy"
COND_THERMAL = "ThermalHealthy"
COND_PROBE = "DeviceProbePassed"

AZURE_CONDITIONS = [COND_READY, COND_PROGRESSING, COND_DEGRADED, COND_DELETING, COND_CREDENTIALS]
MI355X_CONDITIONS = [COND_READY, COND_PROGRESSING, COND_DEGRADED, COND_DELETING,
                     COND_XGMI, COND_ECC, COND_THERMAL, COND_PROBE]

# Mi355xJob condition types (Kubeflow JobCreated/JobRunning/JobRestarting/JobSucceeded/JobFailed,
# plus the Volcano-style gang placement as Scheduled).
COND_SCHEDULED = "Scheduled"
COND_RUNNING = "Running"
COND_RESTARTING = "Restarting"
COND_SUCCEEDED = "Succeeded"
COND_FAILED = "Failed"
COND_SUSPENDED = "Suspended"
JOB_CONDITIONS = [COND_SCHEDULED, COND_RUNNING, COND_RESTARTING, COND_SUCCEEDED, COND_FAILED,
                  COND_SUSPENDED]

AZURE_CREDENTIAL_KEYS = ["AZURE_CLIENT_ID", "AZURE_CLIENT_SECRET", "AZURE_TENANT_ID",
                         "AZURE_SUBSCRIPTION_ID"]  # README.md:108

_S = {"type": "string"}
_I32 = {"type": "integer", "format": "int32"}
_I64 = {"type": "integer", "format": "int64"}
_B = {"type": "boolean"}

CONDITION_SCHEMA = {
    "type": "object",
    "required": ["type", "status", "lastTransitionTime", "reason", "message"],
    "properties": {
        "type": {"type": "string", "maxLength": 316,
                 "pattern": r"^([a-z0-9]([-a-z0-9]*[a-z0-9])?(\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*/)?(([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9])$"},
        "status": {"type": "string", "enum": ["True", "False", "Unknown"]},
        "observedGeneration": {"type": "integer", "format": "int64", "minimum": 0},
        "lastTransitionTime": {"type": "string", "format": "date-time"},
        "reason": {"type": "string", "maxLength": 1024, "minLength": 1,
                   "pattern": r"^[A-Za-z]([A-Za-z0-9_,:]*[A-Za-z0-9_])?$"},
        "message": {"type": "string", "maxLength": 32768},
    },
}

CONDITIONS_FIELD = {
    "type": "array",
    "items": CONDITION_SCHEMA,
    "x-kubernetes-list-type": "map",
    "x-kubernetes-list-map-keys": ["type"],
}

# ---------------------------------------------------------------- AzureVmPool (README.md:92-128)
AZURE_SPEC = {
    "type": "object",
    "description": "AzureVmPoolSpec defines the desired state of AzureVmPool (README.md:92-110).",
    "required": ["replicas", "resourceGroupName", "location", "vmSize", "vnetName", "subnetName",
                 "imageReference", "azureCredentialSecret"],
    "properties": {
        "replicas": {**_I32, "minimum": 0, "description": "Desired number of VM instances."},
        "resourceGroupName": _S,
        "location": _S,
        "vmSize": {**_S, "description": "e.g. Standard_NC4as_T4_v3"},
        "vnetName": _S,
        "subnetName": _S,
        "imageReference": {
            "type": "object",
            "required": ["publisher", "offer", "sku", "version"],
            "properties": {"publisher": _S, "offer": _S, "sku": _S, "version": _S},
        },
        "azureCredentialSecret": {**_S, "description": "Secret with AZURE_CLIENT_ID, "
                                  "AZURE_CLIENT_SECRET, AZURE_TENANT_ID, AZURE_SUBSCRIPTION_ID."},
    },
}

AZURE_STATUS = {
    "type": "object",
    "properties": {
        "observedGeneration": _I64,
        "readyReplicas": _I32,
        "replicas": _I32,
        "vms": {"type": "array", "items": _S},
        "conditions": CONDITIONS_FIELD,
    },
}

# ---------------------------------------------------------------- Mi355xPool
DEVICE_STATUS = {
    "type": "object",
    "required": ["uuid"],
    "properties": {
        "uuid": _S,
        "hipUUID": _S,
        "bdf": _S,
        "index": _I32,
        "node": _S,
        "renderNode": _S,
        "kfdNode": _I32,
        # Unknown: the node's agent does not answer; the entry is its last observation
        "health": {"type": "string", "enum": ["Healthy", "Unhealthy", "Draining", "Probing",
                                              "Unknown"]},
        "reasons": {"type": "array", "items": _S},
        "advertised": _B,
        "pods": {"type": "array", "items": _S},
        "claimedAt": _S,
        "partition": {"type": "object", "properties": {"compute": _S, "memory": _S}},
        "probe": {
            "type": "object",
            "properties": {
                "passed": _B,
                "hbmGBps": {"type": "number"},
                "mfmaTflops": {"type": "number"},
                "xgmiGBps": {"type": "number"},
                "cusVerified": _I32,
                "cusExpected": _I32,
                "ms": {"type": "number"},
                "backend": _S,
                "message": _S,
            },
        },
        "xgmi": {
            "type": "object",
            "description": "xGMI link coverage of this GPU: how many of its pairs with the node's "
                           "other GPUs the agent's peer-copy rings (claim-time checks and idle "
                           "rechecks, in an order rotating to unchecked pairs) have verified, "
                           "which peers failed or could not be checked.",
            "properties": {"pairsCovered": _I32, "pairsTotal": _I32,
                           "failedPeers": {"type": "array", "items": _S},
                           "unavailablePeers": {"type": "array", "items": _S},
                           "lastCheckedAt": _S, "peerCheckUnavailable": _B},
        },
        "sharing": {
            "type": "object",
            "description": "Slot isolation of a shared GPU (spec.sharing): the enforced per-slot "
                           "HBM budget (never above a fair share of the HBM the agent leaves "
                           "free), and per slot its CU-mask bits and the XCDs they land on "
                           "(cuLayout striped: the same number of CUs on every XCD; slots share "
                           "the XCDs' L2s — L2 isolation takes a compute partition).",
            "properties": {"replicasPerGPU": _I32, "hbmBytesPerSlot": _I64,
                           "cuLayout": {"type": "string", "enum": ["striped"]},
                           "cuPerSlot": _I32, "xcds": _I32,
                           "slotCUMasks": {"type": "array", "items": _S},
                           "slotXcds": {"type": "array", "items": _S}},
        },
        "hbmCoverage": {
            "type": "object",
            "description": "The agent's HBM scrubber on this GPU (rotating pattern-test windows "
                           "over all free HBM while the GPU was idle): completed full sweeps, "
                           "fraction of the current sweep, swept span in bytes.",
            "properties": {"passes": _I64, "fraction": {"type": "number"}, "span": _I64,
                           "cursor": _I64, "lastFullSweepAt": {"type": "number"},
                           "lastBadBits": _I64},
        },
    },
}

MI355X_SPEC = {
    "type": "object",
    "description": "Desired state of a pool of MI355X (gfx950) GPUs on one node (or up to "
                   "spec.maxNodes nodes).",
    "required": ["replicas"],
    # cross-field rules the apiserver enforces at admission (CEL); the manager checks the same
    # in native/src/api/api.cc and reports InvalidSpec for objects written before a rule existed
    "x-kubernetes-validations": [
        {"rule": "!has(self.sharing) || !has(self.sharing.cuPerSlot) || "
                 "self.sharing.cuPerSlot == 0 || self.sharing.cuPerSlot * "
                 "(has(self.sharing.replicasPerGPU) ? self.sharing.replicasPerGPU : 1) <= 256",
         "message": "sharing.cuPerSlot x sharing.replicasPerGPU must not exceed the GPU's 256 CUs"},
        {"rule": "!has(self.sharing) || !has(self.sharing.cuPerSlot) || "
                 "self.sharing.cuPerSlot == 0 || self.sharing.cuPerSlot >= "
                 "(has(self.partition) && has(self.partition.compute) ? "
                 "(self.partition.compute == 'CPX' ? 1 : self.partition.compute == 'QPX' ? 2 : "
                 "self.partition.compute == 'DPX' ? 4 : 8) : 8)",
         "message": "sharing.cuPerSlot must be 0 or at least one CU per XCD of the partition "
                    "(8 on SPX): a CU mask that leaves an XCD empty is not applied"},
        {"rule": "!has(self.autoscale) || !has(self.autoscale.minReplicas) || "
                 "!has(self.autoscale.maxReplicas) || "
                 "self.autoscale.minReplicas <= self.autoscale.maxReplicas",
         "message": "autoscale.minReplicas must not exceed autoscale.maxReplicas"},
    ],
    "properties": {
        "replicas": {**_I32, "minimum": 0, "maximum": 1024,
                     "description": "Number of healthy GPUs to claim, probe and advertise."},
        "nodeName": {**_S, "description": "Pin the pool to one node (else nodeSelector/any)."},
        "nodeSelector": {"type": "object", "additionalProperties": _S},
        "maxNodes": {**_I32, "minimum": 1, "maximum": 64, "default": 1,
                     "description": "How many nodes the pool may span (like the reference's pool "
                                    "of N VMs). 1 keeps every GPU of the pool on one xGMI-connected "
                                    "node; above 1 a scale-up that no single node fits is split "
                                    "across nodes (fewest nodes first, all-or-nothing per pass)."},
        "resourceName": {**_S, "default": DEFAULT_RESOURCE,
                         "pattern": r"^[a-z0-9.-]+/[a-z0-9.-]+$",
                         "description": "Extended resource the device plugin advertises "
                                        "this pool's GPUs under."},
        "topologyPolicy": {"type": "string", "enum": ["xgmi-packed", "any"],
                           "default": "xgmi-packed"},
        "partition": {
            "type": "object",
            "default": {},
            "properties": {
                "compute": {"type": "string", "enum": ["Any", "SPX", "DPX", "QPX", "CPX"],
                            "default": "Any"},
                "memory": {"type": "string", "enum": ["Any", "NPS1", "NPS2", "NPS4", "NPS8"],
                           "default": "Any"},
            },
        },
        "sharing": {
            "type": "object",
            "default": {},
            "description": "GPU sharing (the HAMi analogue of the reference platform, "
                           "GPU调度平台搭建.md:289-298): every GPU of the pool is advertised as "
                           "replicasPerGPU devices of resourceName, so that many pods share it. "
                           "hbmBytesPerSlot / cuPerSlot isolate the sharers: the device plugin "
                           "loads libgpupool_share.so into each pod (HSA_TOOLS_LIB), which caps "
                           "the pod's HBM allocations per GPU at hbmBytesPerSlot (hipMalloc & co "
                           "fail with hipErrorOutOfMemory past it, hipMemGetInfo reports the "
                           "budget) and confines its waves to cuPerSlot CUs, disjoint from the "
                           "other slots of the GPU and spread evenly over its XCDs (a kernel's "
                           "workgroups are dealt to every XCD, so a slot needs CUs on each: "
                           "cuPerSlot must be at least the partition's XCD count, 8 on SPX). "
                           "Without them the sharers are only "
                           "time-sliced. A GPU is drained and released only when every pod on "
                           "any of its slots is gone.",
            "properties": {
                "replicasPerGPU": {**_I32, "minimum": 1, "maximum": 64, "default": 1},
                "hbmBytesPerSlot": {**_I64, "minimum": 0, "default": 0,
                                    "description": "HBM budget of one slot in bytes (0 = no "
                                                   "budget)."},
                "cuPerSlot": {**_I32, "minimum": 0, "maximum": 256, "default": 0,
                              "description": "Compute units reserved for one slot (0 = all; "
                                             "cuPerSlot x replicasPerGPU <= 256)."},
                "overBudgetAction": {"type": "string", "enum": ["Flag", "Evict"],
                                     "default": "Flag",
                                     "description": "What the node agent does about a pod whose "
                                                    "VRAM on a GPU (amdsmi / DRM fdinfo, outside "
                                                    "the pod) exceeds its slots' HBM budget — a "
                                                    "pod in which libgpupool_share.so is not in "
                                                    "force: Flag (metric + Node event) or Evict "
                                                    "(after 2 consecutive over-budget samples the "
                                                    "pod is evicted through the API, with an "
                                                    "Event)."},
            },
        },
        "health": {
            "type": "object",
            "default": {},
            "properties": {
                "maxUncorrectableECC": {**_I64, "minimum": 0, "default": 0,
                                        "description": "Uncorrectable ECC errors tolerated "
                                                       "since claim (delta, not absolute)."},
                "maxCorrectableECC": {**_I64, "minimum": 0, "default": 100000,
                                      "description": "Correctable ECC errors tolerated "
                                                     "since claim."},
                "requireAllXGMILinks": {**_B, "default": True},
                "minXGMILinksUp": {**_I32, "minimum": 0, "maximum": 8, "default": 7},
                "thermal": {"type": "string", "default": "belowCritical",
                            "enum": ["belowCritical", "belowEmergency", "ignore"]},
                "thermalMarginC": {**_I32, "minimum": 0, "default": 0},
                "maxRetiredPages": {**_I64, "minimum": 0, "default": 64,
                                    "description": "HBM pages the driver has retired after "
                                                   "uncorrectable errors (absolute, "
                                                   "amdsmi_get_gpu_bad_page_info). Above it the "
                                                   "GPU is unhealthy and never claimed "
                                                   "(HBMRetiredPages)."},
                "maxPendingPages": {**_I64, "minimum": 0, "default": 0,
                                    "description": "Bad HBM pages still awaiting retirement "
                                                   "(HBMPendingRetirement)."},
                "maxLifetimeUncorrectableECC": {**_I64, "minimum": 0,
                                                "description": "Optional limit on the device's "
                                                               "lifetime uncorrectable ECC count "
                                                               "(absolute; unset = only the "
                                                               "delta since claim counts)."},
            },
        },
        "drain": {
            "type": "object",
            "default": {},
            "properties": {
                "gracePeriodSeconds": {**_I64, "minimum": 0, "default": 30},
                "evict": {**_B, "default": True},
                "timeoutSeconds": {**_I64, "minimum": 0, "default": 300},
            },
        },
        "probe": {
            "type": "object",
            "default": {},
            "properties": {
                "enabled": {**_B, "default": True},
                "hbmBytes": {**_I64, "minimum": 1 << 20, "maximum": 64 << 30,
                             "default": 1 << 30},
                "mfma": {**_B, "default": True},
                "minHbmGBps": {"type": "number", "minimum": 0, "default": 0,
                               "description": "Performance floor: a GPU whose probe measures "
                                              "less HBM write+read bandwidth (GB/s) fails "
                                              "DeviceProbePassed (0 = off; MI355X measures "
                                              "~4900 with the default 1 GiB probe)."},
                "xgmiPeerCheck": {**_B, "default": True,
                                  "description": "For pools of 2+ GPUs: each GPU copies a "
                                                 "pattern to the next one over xGMI "
                                                 "(hipMemcpyPeer, ring order) and the receiver "
                                                 "verifies every bit; adds link GB/s to the "
                                                 "probe result."},
                "minXgmiGBps": {"type": "number", "minimum": 0, "default": 0,
                                "description": "Floor for the peer-copy bandwidth of the "
                                               "xGMI check (0 = off)."},
                "recheckSeconds": {**_I32, "minimum": 0, "default": 0,
                                   "description": "Re-run the probe on claimed GPUs that have "
                                                  "no pod every this many seconds (0 = only at "
                                                  "claim time); a failure is handled like any "
                                                  "health fault (DeviceProbePassed, replace)."},
                "minMfmaTflops": {"type": "number", "minimum": 0, "default": 0,
                                  "description": "Performance floor for the probe's 4096^3 bf16 "
                                                 "MFMA GEMM in TFLOP/s (0 = off; MI355X "
                                                 "measures ~1200)."},
                "timeoutSeconds": {"type": "number", "minimum": 0.1, "maximum": 600,
                                   "default": 10,
                                   "description": "Deadline of one GPU's claim-time probe, "
                                                  "including any wait for its (re)starting "
                                                  "probe helper. The probe runs in a helper "
                                                  "process per GPU: past the deadline the "
                                                  "helper is killed and the GPU fails "
                                                  "DeviceProbePassed (ProbeTimeout); a helper "
                                                  "that dies mid-probe fails it as "
                                                  "ProbeCrashed. The xGMI peer ring "
                                                  "(xgmiPeerCheck) has its own deadline of "
                                                  "min(this, 3 s). A claim is answered within "
                                                  "the sum of the two; a GPU still probing "
                                                  "past it plus 5 s is reported probeOverdue "
                                                  "and replaced."},
            },
        },
        "replacePolicy": {"type": "string", "enum": ["Replace", "Keep"], "default": "Replace"},
        "autoscale": {
            "type": "object",
            "description": "Demand-driven replicas (an HPA-style writer of spec.replicas through "
                           "the scale subresource): demand = GPUs of this pool's resourceName "
                           "requested by live pods + waiting or reserved Mi355xJob gangs, clamped "
                           "to [minReplicas, maxReplicas]. Scale-up is immediate; scale-down waits "
                           "until demand has stayed lower for scaleDownDelaySeconds, and only idle "
                           "GPUs are released (drain picks pod-free GPUs first).",
            "properties": {
                "enabled": {**_B, "default": False},
                "minReplicas": {**_I32, "minimum": 0, "maximum": 1024, "default": 0},
                "maxReplicas": {**_I32, "minimum": 0, "maximum": 1024, "default": 8},
                "scaleDownDelaySeconds": {**_I64, "minimum": 0, "default": 300},
            },
        },
    },
}

MI355X_STATUS = {
    "type": "object",
    "properties": {
        "observedGeneration": _I64,
        "replicas": _I32,
        "readyReplicas": _I32,
        "nodeName": _S,
        "nodes": {"type": "array", "items": _S,
                  "description": "Every node holding GPUs of the pool (maxNodes > 1)."},
        "selector": _S,
        "allocatable": {**_I32, "description": "Devices of resourceName the ready GPUs offer "
                                                "(readyReplicas x sharing.replicasPerGPU)."},
        "devices": {"type": "array", "items": DEVICE_STATUS},
        "conditions": CONDITIONS_FIELD,
        "lastReconcileTime": _S,
    },
}

# ---------------------------------------------------------------- Mi355xJob
# The GoHai platform's training-job path (reference GPU调度平台搭建.md:638-675 Volcano Job with
# `minAvailable`/`queue`/`restartPolicy: OnFailure`, :300-306 Kubeflow Training Operator whose
# `PET_*` env the workload reads at :623) as one MI355X-native kind: a gang of pods, each asking
# for `gpusPerReplica` pool GPUs, placed all-or-nothing and wired for torchrun / RCCL.
MI355X_JOB_SPEC = {
    "type": "object",
    "description": "A gang-scheduled distributed training job on pool-advertised MI355X GPUs.",
    "required": ["replicas", "template"],
    "x-kubernetes-validations": [
        {"rule": "!has(self.minAvailable) || self.minAvailable <= self.replicas",
         "message": "minAvailable must not exceed replicas"},
    ],
    "properties": {
        "replicas": {**_I32, "minimum": 1, "maximum": 1024,
                     "description": "Worker pods (torchrun nnodes); placed all-or-nothing."},
        "minAvailable": {**_I32, "minimum": 1, "maximum": 1024,
                         "description": "Elastic gang (Volcano minAvailable): start with as many "
                                        "workers as fit, but at least this many (default: "
                                        "replicas). The attempt's world size is then the number "
                                        "placed (status.workers), handed to PET_NNODES / "
                                        "WORLD_SIZE."},
        "gpusPerReplica": {**_I32, "minimum": 0, "maximum": 64, "default": 1,
                           "description": "GPUs per pod (torchrun nproc-per-node)."},
        "resourceName": {**_S, "pattern": r"^[a-z0-9.-]+/[a-z0-9.-]+$",
                         "description": "Extended resource to request (default: the poolRef's, "
                                        "else amd.com/gpu)."},
        "poolRef": {**_S, "description": "Mi355xPool in this namespace whose GPUs the job "
                                         "uses: its resourceName and node."},
        "nodeSelector": {"type": "object", "additionalProperties": _S},
        "queue": {**_S, "default": "default",
                  "description": "Jobs of one queue are placed strictly in (priority desc, "
                                 "creation) order, so a large gang cannot be starved."},
        "priority": {**_I32, "default": 0},
        "preemptionPolicy": {"type": "string", "enum": ["Never", "PreemptLowerPriority"],
                             "default": "Never",
                             "description": "PreemptLowerPriority: when the gang does not fit, "
                                            "stop running jobs of strictly lower priority (same "
                                            "resource) until it does; victims go back to the queue "
                                            "without using their backoffLimit."},
        "suspend": {**_B, "default": False,
                    "description": "true stops the gang and frees its GPUs (phase Suspended); "
                                   "false resumes it through the queue. Not a restart."},
        "restartPolicy": {"type": "string", "enum": ["OnFailure", "Never"],
                          "default": "OnFailure",
                          "description": "OnFailure: a failed or lost pod restarts the whole "
                                         "gang (DDP ranks cannot rejoin alone)."},
        "backoffLimit": {**_I32, "minimum": 0, "default": 3},
        "activeDeadlineSeconds": {**_I64, "minimum": 0, "default": 0,
                                  "description": "0 = no deadline."},
        "ttlSecondsAfterFinished": {**_I64, "minimum": -1, "default": -1,
                                    "description": "Delete the job this long after it "
                                                   "finished (-1 = keep)."},
        "cleanPodPolicy": {"type": "string", "enum": ["Running", "All", "None"],
                           "default": "Running",
                           "description": "Pods deleted when the job finishes."},
        "successPolicy": {"type": "string", "enum": ["AllWorkers", "Rank0"],
                          "default": "AllWorkers"},
        "masterPort": {**_I32, "minimum": 1, "maximum": 65535, "default": 29500},
        "checkpointDir": {**_S, "description": "Shared directory (e.g. the workspace PVC) passed to "
                                               "every worker as GPUPOOL_CHECKPOINT_DIR: a gang "
                                               "restarted after a failure or preemption resumes "
                                               "from the last checkpoint instead of step 0."},
        "template": {"type": "object", "x-kubernetes-preserve-unknown-fields": True,
                     "description": "Pod template (metadata + spec) of every worker."},
    },
}

MI355X_JOB_STATUS = {
    "type": "object",
    "properties": {
        "observedGeneration": _I64,
        "phase": {"type": "string",
                  "enum": ["Pending", "Running", "Restarting", "Suspended", "Succeeded",
                           "Failed"]},
        "replicas": _I32,
        "workers": {**_I32, "description": "workers placed for the current attempt"},
        "active": _I32,
        "succeeded": _I32,
        "failed": _I32,
        "restarts": _I32,
        "preemptions": _I32,
        "lastPreemption": {**_S, "description": "preempted-by annotation value last acted on"},
        "preempting": {"type": "array", "items": _S,
                       "description": "jobs this one preempted; its pods wait for their GPUs"},
        "attempt": _I32,
        "masterAddr": _S,
        "resourceName": {**_S, "description": "extended resource the pods request (resolved "
                                             "from poolRef at placement)"},
        "startTime": _S,
        "completionTime": _S,
        "placement": {"type": "array", "items": {
            "type": "object",
            "properties": {"index": _I32, "node": _S,
                           "created": {**_B, "description": "pod exists; until then the slot "
                                                            "is a reservation"}}}},
        "replicaStatuses": {"type": "array", "items": {
            "type": "object",
            "properties": {"index": _I32, "pod": _S, "node": _S, "phase": _S, "podIP": _S,
                           "exitCode": _I32, "devices": _S, "message": _S}}},
        "conditions": CONDITIONS_FIELD,
    },
}

# ---------------------------------------------------------------- Mi355xQueue
# Volcano's Queue (the `queue: default` a job names, reference GPU调度平台搭建.md:650; Volcano install
# :275-287) as a cluster-scoped kind: a GPU capability per extended resource, an Open/Closed state
# and whether other queues' higher-priority jobs may preempt its jobs. The queue named "default"
# is implicit (unlimited, open) until an object of that name exists.
MI355X_QUEUE_SPEC = {
    "type": "object",
    "description": "A job queue: GPU capability, admission state and reclaim policy.",
    "properties": {
        "capability": {"type": "object", "additionalProperties": {**_I64, "minimum": 0},
                       "description": "Max GPUs per extended resource (e.g. amd.com/gpu: 16) "
                                      "that this queue's placed jobs may hold together."},
        "state": {"type": "string", "enum": ["Open", "Closed"], "default": "Open",
                  "description": "Closed: no new gang placements; running jobs continue."},
        "reclaimable": {**_B, "default": True,
                        "description": "Jobs of this queue may be preempted by higher-priority "
                                       "PreemptLowerPriority jobs of other queues."},
    },
}

MI355X_QUEUE_STATUS = {
    "type": "object",
    "properties": {
        "observedGeneration": _I64,
        "state": _S,
        "pending": _I32,
        "running": _I32,
        "suspended": _I32,
        "completed": _I32,
        "failed": _I32,
        "allocated": {"type": "object", "additionalProperties": _I64,
                      "description": "GPUs held by placed jobs, per extended resource"},
        "conditions": CONDITIONS_FIELD,
    },
}

KINDS = {
    "AzureVmPool": {
        "plural": "azurevmpools",
        "singular": "azurevmpool",
        "shortNames": ["avp"],
        "spec": AZURE_SPEC,
        "status": AZURE_STATUS,
        "printerColumns": [
            {"name": "Desired", "type": "integer", "jsonPath": ".spec.replicas"},
            {"name": "Ready", "type": "integer", "jsonPath": ".status.readyReplicas"},
            {"name": "Age", "type": "date", "jsonPath": ".metadata.creationTimestamp"},
        ],
        "conditions": AZURE_CONDITIONS,
    },
    "Mi355xPool": {
        "plural": "mi355xpools",
        "singular": "mi355xpool",
        "shortNames": ["mxp"],
        "spec": MI355X_SPEC,
        "status": MI355X_STATUS,
        "printerColumns": [
            {"name": "Desired", "type": "integer", "jsonPath": ".spec.replicas"},
            {"name": "Ready", "type": "integer", "jsonPath": ".status.readyReplicas"},
            {"name": "Node", "type": "string", "jsonPath": ".status.nodeName"},
            {"name": "Status", "type": "string",
             "jsonPath": ".status.conditions[?(@.type==\"Ready\")].reason"},
            {"name": "Age", "type": "date", "jsonPath": ".metadata.creationTimestamp"},
        ],
        "conditions": MI355X_CONDITIONS,
    },
    "Mi355xJob": {
        "plural": "mi355xjobs",
        "singular": "mi355xjob",
        "shortNames": ["mxj"],
        "spec": MI355X_JOB_SPEC,
        "status": MI355X_JOB_STATUS,
        "printerColumns": [
            {"name": "Replicas", "type": "integer", "jsonPath": ".spec.replicas"},
            {"name": "GPUs", "type": "integer", "jsonPath": ".spec.gpusPerReplica"},
            {"name": "Active", "type": "integer", "jsonPath": ".status.active"},
            {"name": "Phase", "type": "string", "jsonPath": ".status.phase"},
            {"name": "Restarts", "type": "integer", "jsonPath": ".status.restarts"},
            {"name": "Age", "type": "date", "jsonPath": ".metadata.creationTimestamp"},
        ],
        "conditions": JOB_CONDITIONS,
        "scale": False,
    },
    "Mi355xQueue": {
        "plural": "mi355xqueues",
        "singular": "mi355xqueue",
        "shortNames": ["mxq"],
        "scope": "Cluster",
        "spec": MI355X_QUEUE_SPEC,
        "status": MI355X_QUEUE_STATUS,
        "printerColumns": [
            {"name": "State", "type": "string", "jsonPath": ".status.state"},
            {"name": "Pending", "type": "integer", "jsonPath": ".status.pending"},
            {"name": "Running", "type": "integer", "jsonPath": ".status.running"},
            {"name": "Allocated", "type": "string", "jsonPath": ".status.allocated"},
            {"name": "Age", "type": "date", "jsonPath": ".metadata.creationTimestamp"},
        ],
        "conditions": [],
        "scale": False,
    },
}


def crd(kind: str) -> dict:
    """Return the apiextensions.k8s.io/v1 CustomResourceDefinition for ``kind``."""
    k = KINDS[kind]
    schema = {
        "type": "object",
        "description": f"{kind} is the Schema for the {k['plural']} API",
        "properties": {
            "apiVersion": _S,
            "kind": _S,
            "metadata": {"type": "object"},
            "spec": copy.deepcopy(k["spec"]),
            "status": copy.deepcopy(k["status"]),
        },
    }
    return {
        "apiVersion": "apiextensions.k8s.io/v1",
        "kind": "CustomResourceDefinition",
        "metadata": {"name": f"{k['plural']}.{GROUP}",
                     "annotations": {"gpupool.amd.com/generated-by": "scripts/gen_manifests.py"}},
        "spec": {
            "group": GROUP,
            "names": {"kind": kind, "listKind": f"{kind}List", "plural": k["plural"],
                      "singular": k["singular"], "shortNames": list(k["shortNames"])},
            "scope": k.get("scope", "Namespaced"),
            "versions": [{
                "name": VERSION,
                "served": True,
                "storage": True,
                "schema": {"openAPIV3Schema": schema},
                "subresources": {"status": {}, **({
                    "scale": {"specReplicasPath": ".spec.replicas",
                              "statusReplicasPath": ".status.readyReplicas"}}
                    if k.get("scale", True) else {})},
                "additionalPrinterColumns": copy.deepcopy(k["printerColumns"]),
            }],
        },
    }


def all_crds() -> list[dict]:
    return [crd(k) for k in KINDS]


def rbac_role() -> dict:
    """ClusterRole the manager needs (the reference's missing 'step four', README.md:162->242)."""
    rules = [
        {"apiGroups": [GROUP], "resources": [k["plural"] for k in KINDS.values()],
         "verbs": ["get", "list", "watch", "create", "update", "patch", "delete"]},
        {"apiGroups": [GROUP], "resources": [k["plural"] + "/status" for k in KINDS.values()],
         "verbs": ["get", "update", "patch"]},
        {"apiGroups": [GROUP], "resources": [k["plural"] + "/finalizers" for k in KINDS.values()],
         "verbs": ["update"]},
        {"apiGroups": [""], "resources": ["secrets"], "verbs": ["get"]},
        {"apiGroups": [""], "resources": ["events"], "verbs": ["create", "patch"]},
        {"apiGroups": [""], "resources": ["pods"],
         "verbs": ["get", "list", "watch", "create", "delete"]},
        {"apiGroups": [""], "resources": ["pods/eviction"], "verbs": ["create"]},
        {"apiGroups": [""], "resources": ["nodes"], "verbs": ["get", "list", "watch", "patch"]},
        {"apiGroups": ["coordination.k8s.io"], "resources": ["leases"],
         "verbs": ["get", "create", "update"]},
        {"apiGroups": [""], "resources": ["resourcequotas"], "verbs": ["get", "list", "watch"]},
    ]
    return {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole",
            "metadata": {"name": "gpupool-manager-role"}, "rules": rules}


AGENT_NAMESPACE = "gpupool-system"


def agent_rbac() -> list[dict]:
    """ServiceAccount + ClusterRole + binding for the node agent DaemonSet: it registers its Node
    (labels, agent-endpoint annotation) and heartbeats the GPUPoolAgentReady/ROCmReady node
    conditions and posts Events on its Node (amdsmi hardware events, HBM sweep failures);
    device/pod facts come from the kubelet's local sockets; it lists pods only to resolve the pod
    UID in a GPU process's cgroup to namespace/name for per-pod accounting, and evicts a pod only
    when its pool asks for it (spec.sharing.overBudgetAction Evict: the pod's VRAM is over its
    slots' HBM budget)."""
    sa = {"apiVersion": "v1", "kind": "ServiceAccount",
          "metadata": {"name": "gpupool-agent", "namespace": AGENT_NAMESPACE}}
    role = {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRole",
            "metadata": {"name": "gpupool-agent-role"},
            # no nodes:create — the kubelet registers the Node; patches are limited to the
            # agent's own Node by the ValidatingAdmissionPolicy below
            "rules": [{"apiGroups": [""], "resources": ["nodes"],
                       "verbs": ["get", "patch"]},
                      {"apiGroups": [""], "resources": ["nodes/status"], "verbs": ["patch"]},
                      {"apiGroups": [""], "resources": ["events"], "verbs": ["create"]},
                      {"apiGroups": [""], "resources": ["pods"], "verbs": ["list"]},
                      {"apiGroups": [""], "resources": ["pods/eviction"], "verbs": ["create"]}]}
    binding = {"apiVersion": "rbac.authorization.k8s.io/v1", "kind": "ClusterRoleBinding",
               "metadata": {"name": "gpupool-agent-rolebinding"},
               "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole",
                           "name": "gpupool-agent-role"},
               "subjects": [{"kind": "ServiceAccount", "name": "gpupool-agent",
                             "namespace": AGENT_NAMESPACE}]}
    return [sa, role, binding, *agent_node_policy()]


AGENT_SA_USER = f"system:serviceaccount:{AGENT_NAMESPACE}:gpupool-agent"
AGENT_OWN_CONDITIONS = ["GPUPoolAgentReady", "ROCmReady"]
AGENT_LABEL_PREFIXES = ["amd.com/", "gpupool.amd.com/"]


def agent_node_policy() -> list[dict]:
    """RBAC cannot say "only your own Node": a ValidatingAdmissionPolicy can. A Node write by the
    agent ServiceAccount is admitted only when (1) the bound token's node claim
    (``authentication.kubernetes.io/node-name``, set on projected tokens of pods since k8s 1.30)
    names that Node, (2) ``spec`` is untouched, (3) in ``status`` nothing but the agent's own
    conditions changed (capacity, allocatable and the kubelet's conditions are the kubelet's), and
    (4) only labels/annotations under the agent's prefixes changed. apiserver-sim enforces the same
    rules natively (store.AgentNodePolicy) when this policy object is present."""
    own = "[" + ", ".join(f"'{t}'" for t in AGENT_OWN_CONDITIONS) + "]"
    pre = "[" + ", ".join(f"'{p}'" for p in AGENT_LABEL_PREFIXES) + "]"

    def unchanged_outside_prefixes(field: str) -> str:
        new, old = f"variables.{field}", f"variables.{field}Old"
        return (f"{old}.all(k, {pre}.exists(p, k.startsWith(p)) || "
                f"(k in {new} && {new}[k] == {old}[k])) && "
                f"{new}.all(k, {pre}.exists(p, k.startsWith(p)) || k in {old})")
    policy = {
        "apiVersion": "admissionregistration.k8s.io/v1", "kind": "ValidatingAdmissionPolicy",
        "metadata": {"name": "gpupool-agent-own-node"},
        "spec": {
            "failurePolicy": "Fail",
            "matchConstraints": {"resourceRules": [{
                "apiGroups": [""], "apiVersions": ["v1"], "operations": ["UPDATE"],
                "resources": ["nodes", "nodes/status"]}]},
            "matchConditions": [{"name": "gpupool-agent",
                                 "expression": f"request.userInfo.username == '{AGENT_SA_USER}'"}],
            "variables": [
                {"name": "nodeClaim",
                 "expression": "'authentication.kubernetes.io/node-name' in request.userInfo.extra"
                               " ? request.userInfo.extra['authentication.kubernetes.io/node-name']"
                               "[0] : ''"},
                {"name": "others",
                 "expression": f"has(object.status.conditions) ? object.status.conditions.filter("
                               f"c, !(c.type in {own})) : []"},
                {"name": "othersOld",
                 "expression": f"has(oldObject.status.conditions) ? oldObject.status.conditions"
                               f".filter(c, !(c.type in {own})) : []"},
                *({"name": f"{f}{sfx}",
                   "expression": f"has({o}.metadata.{f}) ? {o}.metadata.{f} : {{}}"}
                  for f in ("labels", "annotations")
                  for sfx, o in (("", "object"), ("Old", "oldObject")))],
            "validations": [
                {"expression": "variables.nodeClaim == object.metadata.name",
                 "reason": "Forbidden",
                 "message": "the gpupool agent may only write the Node it runs on"},
                {"expression": "object.?spec == oldObject.?spec", "reason": "Forbidden",
                 "message": "the gpupool agent may not change Node spec"},
                {"expression": "object.status.?capacity == oldObject.status.?capacity && "
                               "object.status.?allocatable == oldObject.status.?allocatable && "
                               "variables.others == variables.othersOld",
                 "reason": "Forbidden",
                 "message": "the gpupool agent may only write its own Node conditions "
                            f"({', '.join(AGENT_OWN_CONDITIONS)})"},
                {"expression": unchanged_outside_prefixes("labels") + " && " +
                               unchanged_outside_prefixes("annotations"),
                 "reason": "Forbidden",
                 "message": "the gpupool agent may only write labels/annotations under "
                            f"{', '.join(AGENT_LABEL_PREFIXES)}"}]}}
    binding = {"apiVersion": "admissionregistration.k8s.io/v1",
               "kind": "ValidatingAdmissionPolicyBinding",
               "metadata": {"name": "gpupool-agent-own-node"},
               "spec": {"policyName": "gpupool-agent-own-node", "validationActions": ["Deny"]}}
    return [policy, binding]
