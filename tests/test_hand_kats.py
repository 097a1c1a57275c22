"""Hand-derived known answers (tests/golden/hand_kats.json) for the paths the survey's
KATs do not cover: LOCAL WITH_START (Q8), semi-global end conventions (Q3, Q10, Q11),
local second-best (Q13), KSW (Q16), banded and the reverse / complement pre-op.  Each
case's derivation is written out in the fixture from the cited reference lines, so it
checks the oracle and the HIP kernels without trusting either (the oracle and the
thread-per-pair kernels are close restatements of each other)."""
import json
import os

import numpy as np
import pytest

import gasal_ffi as G
import helpers
import oracle as O

with open(os.path.join(helpers.GOLDEN, "hand_kats.json")) as _f:
    CASES = json.load(_f)["cases"]


def _run(mod, make, case, engine=None):
    b = G.Batch.from_pairs([case["q"]], [case["t"]])
    qo = np.array([case["q_op"]], np.uint8) if "q_op" in case else None
    to = np.array([case["t_op"]], np.uint8) if "t_op" in case else None
    seed = np.array([case["seed"]], np.uint32) if "seed" in case else None
    p = make(**case["params"])
    if engine is None:
        return O.align(b, p, q_ops=qo, t_ops=to, seed_scores=seed)
    return engine.align_host(b, p, q_ops=qo, t_ops=to, seed_scores=seed)


def _check(out, case):
    for k, v in case["expect"].items():
        assert int(out[k][0]) == v, f"{case['name']}: {k} = {int(out[k][0])}, expected {v} ({case['derivation']})"


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_oracle_hand_kats(case):
    _check(_run(O, O.make_params, case), case)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_gpu_hand_kats(engine, case):
    _check(_run(G, G.make_params, case, engine), case)
