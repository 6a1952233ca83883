"""Trace loader -> SoA and the HBM-resident anchor path.

Pinned against the reference's own loader: tests/golden/make_trace_sample.py ran
TraceBasedApplicationGenerator (alibaba/runner.py:54-136) on a 400-job subset of the bundled
trace and recorded, per container, its demand and the predecessor-task list cost_aware counts
(scheduler/cost_aware.py:51). ``pivot_place.trace`` must reproduce both exactly; the gpu tests
then resolve anchors through DeviceTrace (pvt_anchor over the resident table, item form) and
compare them with the CPU restatement and with the reference's Counter expression.
"""
import collections
import gzip
import json
import os

import numpy as np
import pytest

from oracle import oracle
from pivot_place import trace

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _ref():
    with gzip.open(os.path.join(GOLDEN, "trace_sample_ref.json.gz"), "rt") as f:
        return json.load(f)


def _trace():
    ref = _ref()
    return trace.load(os.path.join(GOLDEN, "jobs_sample.yaml.gz"),
                      output_size_scale_factor=ref["output_size_scale_factor"],
                      n_apps=ref["n_apps"]), ref


def test_trace_matches_reference_loader():
    tr, ref = _trace()
    assert tr.app_ids == [a["id"] for a in ref["apps"]]
    c = 0
    for a, app in enumerate(ref["apps"]):
        assert tr.app_off[a] == c
        for cont in app["containers"]:
            assert tr.cont_ids[c] == cont["id"] and tr.cont_app[c] == a
            assert tr.cpus[c] == cont["cpus"] and tr.mem[c] == cont["mem"]
            assert tr.output_size[c] == cont["output_size"] and tr.runtime[c] == cont["runtime"]
            assert tr.n_inst[c] == cont["instances"]
            want = [tr.inst_base[tr.container_index(a, pid)] + j for pid, j in cont["preds"]]
            got = tr.pinst[tr.pinst_off[c]:tr.pinst_off[c + 1]].tolist()
            assert got == want, (a, cont["id"])
            c += 1
    assert c == tr.n_containers
    assert tr.n_instances == sum(cont["instances"] for app in ref["apps"]
                                 for cont in app["containers"])


def test_trace_edge_cases():
    jobs = [
        {"id": "b", "submit_time": 5, "tasks": [
            {"id": 1, "cpus": 1, "mem": 0.5, "runtime": 3, "n_instances": 2, "dependencies": []},
            {"id": 2, "cpus": 2, "mem": 0.25, "runtime": 4, "n_instances": 3,
             "dependencies": [1, 1]},          # a repeated dependency adds one edge
            {"id": 1, "cpus": 3, "mem": 0.5, "runtime": 3, "n_instances": 1,
             "dependencies": []}]},            # redefinition: first position, last value
        {"id": "a", "submit_time": 5, "tasks": []},
        {"id": "c", "submit_time": 1, "tasks": [
            {"id": 9, "cpus": 1, "mem": 1.0, "runtime": 1, "n_instances": 1, "dependencies": []}]},
    ]
    tr = trace.from_jobs(jobs)
    assert tr.app_ids == ["c", "b", "a"]          # by submit time, ties in file order
    assert tr.cont_ids == ["9", "1", "2"] and tr.cpus.tolist() == [1, 3, 2]
    assert tr.n_inst.tolist() == [1, 1, 3]
    assert tr.pinst_off.tolist() == [0, 0, 0, 1] and tr.pinst.tolist() == [1]
    assert trace.from_jobs(jobs, n_apps=1).app_ids == ["c"]


def _round_placements(tr, rng, H):
    inst_host = rng.integers(-1, H, size=tr.n_instances).astype(np.int32)
    inst_host[rng.random(tr.n_instances) < 0.5] = rng.integers(0, 3)   # many ties on 3 hosts
    return inst_host


@pytest.mark.gpu
def test_gpu_device_trace_anchors(engine):
    tr, _ = _trace()
    H = 1000
    rng = np.random.default_rng(17)
    zone = (np.arange(H) % 31).astype(np.int32)
    dt = trace.DeviceTrace(tr, zone, engine)
    inst_host = _round_placements(tr, rng, H)
    dt.record(np.arange(tr.n_instances), inst_host)
    ready = rng.permutation(tr.n_containers)[:700].astype(np.int32)
    ready = np.concatenate([ready, ready[:50]])   # rows may repeat within a call
    mode, az = dt.anchors(ready)
    mode, az = mode.cpu().numpy(), az.cpu().numpy()
    want = oracle.anchor(tr.pinst_off, tr.pinst, zone, H, inst_host=inst_host)
    assert want[2] == 0
    assert np.array_equal(mode, want[0][ready]) and np.array_equal(az, want[1][ready])
    for i, c in enumerate(ready[:200]):
        L = inst_host[tr.pinst[tr.pinst_off[c]:tr.pinst_off[c + 1]]].tolist()
        if L:
            m = max(collections.Counter(L).items(), key=lambda x: x[1])[0]
            assert mode[i] == m
    # a second round: placements of some instances change, anchors follow
    sel = rng.choice(tr.n_instances, size=2000, replace=False)
    newh = rng.integers(0, H, size=2000).astype(np.int32)
    dt.record(sel, newh)
    inst_host[sel] = newh
    mode, az = dt.anchors(ready)
    want = oracle.anchor(tr.pinst_off, tr.pinst, zone, H, inst_host=inst_host)
    assert np.array_equal(mode.cpu().numpy(), want[0][ready])
    assert np.array_equal(az.cpu().numpy(), want[1][ready])


@pytest.mark.gpu
def test_gpu_device_trace_rejects_bad_rows(engine):
    tr, _ = _trace()
    zone = np.zeros(10, dtype=np.int32)
    dt = trace.DeviceTrace(tr, zone, engine)
    with pytest.raises(RuntimeError, match="EINVAL"):
        dt.anchors([0, tr.n_containers])
