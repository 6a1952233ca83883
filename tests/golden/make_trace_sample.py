#!/usr/bin/env python3
"""Trace-loader fixtures from the REFERENCE's own loader (test-only; runs in the build container).

Writes
* ``jobs_sample.yaml.gz``: the first 400 jobs of the bundled
  alibaba/jobs/jobs-5000-200-172800-259200.yaml, byte for byte (a data subset of the trace the
  reference ships; job boundaries are the top-level ``- `` lines);
* ``trace_sample_ref.json.gz``: what the reference's ``TraceBasedApplicationGenerator``
  (alibaba/runner.py:54-136) builds from that subset with output_size_scale_factor 1000 and
  n_apps 300: applications in submission order, per container (``Application.containers``
  order) its cpus / mem / output_size / runtime / instances, and the list the cost_aware policy
  iterates — ``[t for p in app.get_predecessors(c.id) for t in p.tasks]``
  (scheduler/cost_aware.py:51) — as (predecessor container id, task index) pairs, after every
  container's ``generate_tasks()`` has run (application/__init__.py:309-315).

The reference runs on ``pivot_place.des`` (the SimPy restatement) with make_golden.py's
compatibility shims (collections.Iterable, yaml Loader). Only the two fixtures travel.
"""
import gzip
import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
SRC = os.path.join(REF, "alibaba", "jobs", "jobs-5000-200-172800-259200.yaml")
N_JOBS, N_APPS, OSF = 400, 300, 1000


def main():
    sys.path.insert(0, os.path.join(ROOT, "pivot-scheduling_amd"))
    sys.path.insert(0, HERE)
    text = open(SRC).read().splitlines(keepends=True)
    starts = [i for i, ln in enumerate(text) if ln.startswith("- ")]
    sub = "".join(text[:starts[N_JOBS]])
    with gzip.open(os.path.join(HERE, "jobs_sample.yaml.gz"), "wt") as f:
        f.write(sub)
    from pivot_place import des
    des.install(force=True)
    import make_golden as mg
    mg._install_compat()
    sys.path.insert(0, REF)
    sys.path.insert(0, os.path.join(REF, "alibaba"))
    import simpy
    from runner import TraceBasedApplicationGenerator
    with tempfile.NamedTemporaryFile("w", suffix=".yaml", delete=False) as tf:
        tf.write(sub)
    env = simpy.Environment()
    gen = TraceBasedApplicationGenerator(env, tf.name, None, OSF, N_APPS)
    os.unlink(tf.name)
    apps = gen.apps
    out = {"n_jobs": N_JOBS, "n_apps": N_APPS, "output_size_scale_factor": OSF, "apps": []}
    for app in apps:
        for c in app.containers:
            list(c.generate_tasks())
    for app in apps[:N_APPS]:
        conts = []
        for c in app.containers:
            preds = [(p.id, int(t.id.split("/")[-1])) for p in app.get_predecessors(c.id)
                     for t in p.tasks]
            conts.append({"id": c.id, "cpus": c.cpus, "mem": c.mem, "output_size": c.output_size,
                          "runtime": c.runtime, "instances": c.instances, "preds": preds})
        out["apps"].append({"id": app.id, "containers": conts})
    with gzip.open(os.path.join(HERE, "trace_sample_ref.json.gz"), "wt") as f:
        json.dump(out, f)
    print("apps", len(out["apps"]), "containers", sum(len(a["containers"]) for a in out["apps"]))


if __name__ == "__main__":
    main()
