"""Condition helpers, exit-code policy and the workload gate.

Ports ``pkg/util/status_test.go``, ``pkg/util/train/train_util_test.go`` and
``pkg/util/workloadgate/workload_gate_test.go``, plus hypothesis properties
of the condition state machine.
"""
import pytest
from hypothesis import given, settings, strategies as st

from kubedl_amd.api import common as c
from kubedl_amd.controllers.workloadgate import is_workload_enable, parse_workloads_enabled


def test_is_succeeded_failed():
    s = c.new_job_status()
    assert not c.is_succeeded(s) and not c.is_failed(s)
    c.update_job_conditions(s, c.JOB_SUCCEEDED, "r", "m")
    assert c.is_succeeded(s)
    s = c.new_job_status()
    c.update_job_conditions(s, c.JOB_FAILED, "r", "m")
    assert c.is_failed(s)


def test_update_job_conditions_sequence():
    s = c.new_job_status()
    c.update_job_conditions(s, c.JOB_CREATED, c.JOB_CREATED_REASON, "created")
    assert [x["type"] for x in s["conditions"]] == ["Created"]
    c.update_job_conditions(s, c.JOB_RUNNING, c.JOB_RUNNING_REASON, "running")
    assert [x["type"] for x in s["conditions"]] == ["Created", "Running"]
    # same type + reason -> no-op
    before = [dict(x) for x in s["conditions"]]
    c.update_job_conditions(s, c.JOB_RUNNING, c.JOB_RUNNING_REASON, "running again")
    assert s["conditions"] == before
    # Restarting replaces Running
    c.update_job_conditions(s, c.JOB_RESTARTING, c.JOB_RESTARTING_REASON, "restarting")
    assert [x["type"] for x in s["conditions"]] == ["Created", "Restarting"]
    c.update_job_conditions(s, c.JOB_RUNNING, c.JOB_RUNNING_REASON, "running")
    assert [x["type"] for x in s["conditions"]] == ["Created", "Running"]
    # Succeeded flips Running to False
    c.update_job_conditions(s, c.JOB_SUCCEEDED, c.JOB_SUCCEEDED_REASON, "done")
    types = {x["type"]: x["status"] for x in s["conditions"]}
    assert types == {"Created": "True", "Running": "False", "Succeeded": "True"}
    assert s["conditions"][-1]["type"] == "Succeeded"


def test_failed_is_final():
    s = c.new_job_status()
    c.update_job_conditions(s, c.JOB_FAILED, c.JOB_FAILED_REASON, "boom")
    c.update_job_conditions(s, c.JOB_RUNNING, c.JOB_RUNNING_REASON, "running")
    assert [x["type"] for x in s["conditions"]] == ["Failed"]


def test_same_status_keeps_transition_time():
    s = c.new_job_status()
    c.update_job_conditions(s, c.JOB_RUNNING, "A", "m", ts="2020-01-01T00:00:00.000000Z")
    c.update_job_conditions(s, c.JOB_RUNNING, "B", "m", ts="2021-01-01T00:00:00.000000Z")
    cond = c.get_condition(s, "Running")
    assert cond["reason"] == "B"
    assert cond["lastTransitionTime"] == "2020-01-01T00:00:00.000000Z"
    assert cond["lastUpdateTime"] == "2021-01-01T00:00:00.000000Z"


@given(st.lists(st.sampled_from(c.CONDITION_TYPES), min_size=1, max_size=30))
@settings(max_examples=200, deadline=None)
def test_condition_invariants(seq):
    s = c.new_job_status()
    failed_at = None
    for i, t in enumerate(seq):
        c.update_job_conditions(s, t, t + "Reason", "m")
        if t == c.JOB_FAILED and failed_at is None:
            failed_at = i
        types = [x["type"] for x in s["conditions"]]
        assert len(types) == len(set(types)), "each condition type appears once"
        true_types = {x["type"] for x in s["conditions"] if x["status"] == "True"}
        assert not ({"Running", "Restarting"} <= true_types)
        if failed_at is not None:
            assert c.is_failed(s)
            assert s["conditions"][-1]["type"] == "Failed"  # nothing is appended after Failed


@pytest.mark.parametrize("code,retry", [
    (0, False), (1, False), (2, False), (126, False), (127, False), (128, False), (139, False),
    (130, True), (137, True), (143, True), (138, True), (3, False), (255, False), (134, False)])
def test_exit_code_policy(code, retry):
    assert c.is_retryable_exit_code(code) is retry


@pytest.mark.parametrize("workloads,enables,enable_all", [
    ("", {}, False),
    ("*", {}, True),
    ("*,foo", {"foo": True}, True),
    ("foo,*", {"foo": True}, True),
    ("foo,a", {"foo": True, "a": True}, False),
    ("foo,-a", {"foo": True, "a": False}, False),
    ("-foo,a", {"foo": False, "a": True}, False),
    ("foo,-*", {"foo": True}, False),
])
def test_parse_workloads_enabled(workloads, enables, enable_all):
    assert parse_workloads_enabled(workloads) == (enables, enable_all)


def test_is_workload_enable_semantics():
    assert is_workload_enable("TFJob", "auto", env={})
    assert not is_workload_enable("TFJob", "auto", crd_installed=lambda k: False, env={})
    assert is_workload_enable("TFJob", "TFJob,PyTorchJob", env={})
    assert not is_workload_enable("XDLJob", "TFJob,PyTorchJob", env={})
    assert is_workload_enable("XDLJob", "*", env={})
    # quirk: presence, not value -> "-TFJob" enables TFJob
    assert is_workload_enable("TFJob", "-TFJob", env={})
    # env only consulted when the flag is not auto
    assert is_workload_enable("XDLJob", "auto", env={"WORKLOADS_ENABLE": "TFJob"})
    assert not is_workload_enable("XDLJob", "", env={"WORKLOADS_ENABLE": "TFJob"})
    assert is_workload_enable("TFJob", "", env={"WORKLOADS_ENABLE": "TFJob"})
