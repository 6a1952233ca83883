"""pivot_place — MI355X (gfx950) placement engine for the PIVOT scheduling simulator.

The hot path of the reference (dcvan24/pivot-scheduling) is a policy's ``schedule(tasks)``:
score every ready-task x host candidate and pick a host per task, committing capacity in
order. This package runs it in hand-written HIP kernels behind a C ABI
(include/pivot_place.h, libpivot_place.so) and keeps the reference's plugin contract in
Python (``pivot_place.policies``).

    from pivot_place.policies import CostAwareGlobalScheduler   # drop-in for the reference's
"""
from ._abi import (PVT_CA_BF, PVT_CA_FF, PVT_OPP, PVT_VBP_BF, PVT_VBP_FF, RoundArrays,  # noqa
                   RoundResult)

__all__ = ["PVT_CA_FF", "PVT_CA_BF", "PVT_OPP", "PVT_VBP_FF", "PVT_VBP_BF", "RoundArrays",
           "RoundResult"]
__version__ = "0.1.0"
