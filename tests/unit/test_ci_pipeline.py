"""The CI/CD pipeline (.gitlab-ci.yml; SURVEY B24, the reference's GitLab stages
build/push/deploy/train at GPU调度平台搭建.md:748-794) is consistent with this repository: every
Make target, file, manifest image line and gpuctl verb it uses exists, images are gated by the
CPU and the MI355X test stages, and credentials never reach argv."""
from __future__ import annotations

import os
import re
import shlex

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _ci() -> dict:
    with open(os.path.join(ROOT, ".gitlab-ci.yml")) as f:
        return yaml.safe_load(f)


def _jobs(ci: dict) -> dict:
    return {k: v for k, v in ci.items() if isinstance(v, dict) and "stage" in v}


def _script(job: dict, ci: dict) -> list[str]:
    base = ci.get(job.get("extends", ""), {}) if isinstance(job.get("extends"), str) else {}
    return list(base.get("before_script", [])) + list(job.get("script", []))


def test_stages_and_gates():
    ci = _ci()
    assert ci["stages"] == ["build", "test", "push", "deploy", "train"]
    jobs = _jobs(ci)
    assert {j["stage"] for j in jobs.values()} == set(ci["stages"])  # no empty stage
    assert set(jobs["push"]["needs"]) >= {"build", "test-cpu", "test-gpu"}
    assert "mi355x" in jobs["test-gpu"]["tags"]
    assert jobs["deploy"]["needs"] == ["push"] and jobs["train"]["needs"] == ["push"]
    assert jobs["train"]["rules"] == [{"if": "$CI_COMMIT_TAG"}]


def test_every_make_target_file_and_gpuctl_verb_exists():
    ci = _ci()
    makefile = open(os.path.join(ROOT, "Makefile")).read()
    targets = set()
    for line in makefile.splitlines():
        m = re.match(r"^([a-zA-Z0-9_ -]+):(?!=)", line)
        if m:
            targets.update(m.group(1).split())
    from gpupool.cli.gpuctl import build_parser
    verbs = set(build_parser()._subparsers._group_actions[0].choices)
    for name, job in _jobs(ci).items():
        for cmd in _script(job, ci):
            words = shlex.split(cmd.split("|")[0].split(">")[0])
            if words[:1] == ["make"]:
                for t in words[1:]:
                    if "=" not in t:
                        assert t in targets, (name, t)
            for i, w in enumerate(words):
                if w in ("-f", "--filename") and i + 1 < len(words) and "$" not in words[i + 1] \
                        and not words[i + 1].endswith("job.yaml"):
                    assert os.path.exists(os.path.join(ROOT, words[i + 1])), (name, words[i + 1])
                if w.startswith(("scripts/", "config/", "deploy/")):
                    assert os.path.exists(os.path.join(ROOT, w)), (name, w)
            if words and words[0] == "bin/gpuctl":
                verb = next(w for w in words[1:] if not w.startswith("-") and "$" not in w
                            and w != "--kubeconfig")
                assert verb in verbs, (name, verb)


def test_deploy_image_substitutions_match_the_manifests():
    ci = _ci()
    for cmd in _jobs(ci)["deploy"]["script"]:
        m = re.match(r'sed -i "s#(image: [^#]+)#[^#]+#" (\S+)', cmd)
        if m:
            assert m.group(1) in open(os.path.join(ROOT, m.group(2))).read(), cmd


def test_registry_password_never_on_the_command_line():
    ci = _ci()
    for name, job in _jobs(ci).items():
        for cmd in _script(job, ci):
            if "docker login" in cmd:
                assert "--password-stdin" in cmd and " -p " not in cmd, (name, cmd)


def test_train_job_template_is_what_the_pipeline_edits():
    import subprocess
    import sys
    out = subprocess.run([sys.executable, "-m", "gpupool.cli", "trainjob", "template"],
                         capture_output=True, text=True, cwd=ROOT, check=True).stdout
    keys = [ln.split(":")[0] for ln in out.splitlines() if ln and not ln.startswith(" ")]
    assert "image" in keys and "title" in keys  # the two lines the train job rewrites
