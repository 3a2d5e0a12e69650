"""gpuctl convert: the reference's Volcano Job (GPU调度平台搭建.md:643-672) and a Kubeflow
PyTorchJob (the training operator it installs, :300-306) as Mi355xJob gangs (gpupool/cli/convert.py)."""
from __future__ import annotations

import copy
import os
import subprocess
import sys

import pytest
import yaml

from gpupool.cli.convert import ConvertError, convert

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF_VCJOB = os.path.join(ROOT, "tests", "fixtures", "foreign", "reference_vcjob.yaml")
PTJ = os.path.join(ROOT, "config", "samples", "foreign", "kubeflow_pytorchjob.yaml")


def test_reference_volcano_job_converts_with_warnings():
    job, warns = convert(yaml.safe_load(open(REF_VCJOB)))
    assert job["apiVersion"] == "compute.my.domain/v1alpha1" and job["kind"] == "Mi355xJob"
    assert job["metadata"]["name"] == "fashion-mnist-job"
    assert job["metadata"]["annotations"]["gpupool.amd.com/converted-from"] == \
        "batch.volcano.sh/v1alpha1/Job"
    s = job["spec"]
    assert s["replicas"] == 1 and s["gpusPerReplica"] == 1 and s["queue"] == "default"
    assert s["restartPolicy"] == "OnFailure" and "minAvailable" not in s  # == replicas
    c = s["template"]["spec"]["containers"][0]
    assert c["command"] == ["bash", "-lc"] and "python train.py" in c["args"][0]
    assert "resources" not in c  # the controller writes the pool's resource itself
    assert "restartPolicy" not in s["template"]["spec"]
    assert s["template"]["spec"]["volumes"] == [
        {"name": "dataset", "persistentVolumeClaim": {"claimName": "fashionmnist-dataset-pvc"}}]
    # what does not carry over is said: the CUDA image, the volume nothing mounts
    assert any("CUDA image" in w for w in warns), warns
    assert any("no container mounts" in w for w in warns), warns
    job2, warns2 = convert(yaml.safe_load(open(REF_VCJOB)), image="rocm/pytorch:latest",
                           pool="train-pool")
    assert job2["spec"]["template"]["spec"]["containers"][0]["image"] == "rocm/pytorch:latest"
    assert job2["spec"]["poolRef"] == "train-pool" and not any("CUDA" in w for w in warns2)


def test_volcano_elastic_gang_retries_and_volume_mounts():
    doc = yaml.safe_load(open(REF_VCJOB))
    doc["spec"].update({"minAvailable": 2, "maxRetry": 5, "ttlSecondsAfterFinished": 60,
                        "volumes": [{"mountPath": "/data", "volumeClaimName": "ds"}]})
    doc["spec"]["tasks"][0]["replicas"] = 4
    job, _ = convert(doc)
    s = job["spec"]
    assert s["replicas"] == 4 and s["minAvailable"] == 2 and s["backoffLimit"] == 5
    assert s["ttlSecondsAfterFinished"] == 60
    pod = s["template"]["spec"]
    assert pod["volumes"] == [{"name": "volcano-vol-0", "persistentVolumeClaim": {"claimName": "ds"}}]
    assert pod["containers"][0]["volumeMounts"] == [{"name": "volcano-vol-0", "mountPath": "/data"}]


def test_volcano_tasks_with_different_templates_are_refused():
    doc = yaml.safe_load(open(REF_VCJOB))
    other = copy.deepcopy(doc["spec"]["tasks"][0])
    other["name"] = "ps"
    other["template"]["spec"]["containers"][0]["args"] = ["python ps.py"]
    doc["spec"]["tasks"].append(other)
    with pytest.raises(ConvertError, match="different pod templates"):
        convert(doc)
    same = copy.deepcopy(doc["spec"]["tasks"][0])
    same["name"] = "train2"
    doc["spec"]["tasks"][1] = same
    assert convert(doc)[0]["spec"]["replicas"] == 2


def test_pytorchjob_master_and_workers_become_one_gang():
    job, warns = convert(yaml.safe_load(open(PTJ)))
    s = job["spec"]
    assert s["replicas"] == 2 and s["gpusPerReplica"] == 1 and s["backoffLimit"] == 2
    assert s["cleanPodPolicy"] == "Running" and s["restartPolicy"] == "OnFailure"
    assert job["metadata"]["annotations"]["gpupool.amd.com/converted-from"] == "kubeflow.org/v1/PyTorchJob"
    assert not warns, warns
    doc = yaml.safe_load(open(PTJ))
    doc["spec"]["pytorchReplicaSpecs"]["Worker"]["replicas"] = 3
    doc["spec"]["elasticPolicy"] = {"minReplicas": 2, "maxReplicas": 4}
    job, _ = convert(doc)
    assert job["spec"]["replicas"] == 4 and job["spec"]["minAvailable"] == 2
    doc["spec"]["pytorchReplicaSpecs"]["Worker"]["template"]["spec"]["containers"][0]["image"] = "x"
    with pytest.raises(ConvertError, match="differ"):
        convert(doc)


def test_gpuctl_convert_cli_prints_the_job_and_warnings():
    r = subprocess.run([sys.executable, "-m", "gpupool.cli", "convert", "-f", REF_VCJOB,
                        "--pool", "p"], capture_output=True, text=True, timeout=60, cwd=ROOT,
                       env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0, r.stderr
    job = yaml.safe_load(r.stdout)
    assert job["kind"] == "Mi355xJob" and job["spec"]["poolRef"] == "p"
    assert "warning: fashion-mnist-job: container trainer: image" in r.stderr
