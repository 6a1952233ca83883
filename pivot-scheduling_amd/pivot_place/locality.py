"""Zone tables of the cross-cloud cluster (reference resources/__init__.py:546-589).

``data/locality.json`` holds the reference's locality.yml as data: the zone list and the
region-pair (cost, bw) table, both in YAML order (tools/extract_data.py writes it). The
reference expands every region pair into its zone pairs and multiplies each bw by
U(.95, 1.05), drawn from numpy's global RNG in that order (resources/__init__.py:580-589).
``zone_tables(seed)`` redoes that with an explicit RandomState(seed), which is the same stream
as ``np.random.seed(seed)`` before the first ``ResourceMetadata()``.
"""
import functools
import json
import os

import numpy as np

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")


@functools.lru_cache(maxsize=None)
def _doc():
    with open(os.path.join(DATA, "locality.json")) as f:
        return json.load(f)


def zone_names():
    """``cloud/region/zone`` strings in locality.yml order (ResourceMetadata.zones)."""
    return ["%s/%s/%s" % (r["cloud"], r["region"], z) for r in _doc()["regions"] for z in r["zones"]]


def zone_tables(seed=0, n_zones=None):
    """(cost, bw) as Z x Z fp64 arrays indexed [src_zone, dst_zone].

    ``n_zones`` keeps the first n zones of YAML order (SURVEY.md §8(d) uses 20); the jitter is
    drawn for all 31 x 31 pairs first, so the kept entries equal the full table's."""
    doc = _doc()
    names = zone_names()
    index = {n: i for i, n in enumerate(names)}
    zones_of = {"%s_%s" % (r["cloud"], r["region"]): ["%s/%s/%s" % (r["cloud"], r["region"], z)
                                                      for z in r["zones"]] for r in doc["regions"]}
    Z = len(names)
    cost = np.full((Z, Z), np.nan)
    bw = np.full((Z, Z), np.nan)
    rs = np.random.RandomState(seed)
    for m in doc["meta"]:
        for sz in zones_of[m["src"]]:
            for dz in zones_of[m["dst"]]:
                i, j = index[sz], index[dz]
                cost[i, j] = m["cost"]
                bw[i, j] = m["bw"] * rs.uniform(.95, 1.05)
    if np.isnan(cost).any() or np.isnan(bw).any():
        raise ValueError("locality.json does not cover every zone pair")
    if n_zones is not None:
        cost, bw = cost[:n_zones, :n_zones].copy(), bw[:n_zones, :n_zones].copy()
    return cost, bw
