"""The CPU oracle against the golden images SwiftShader rendered from the
reference GLSL (tests/golden/make_goldens.py) -- pins the oracle."""
import glob
import json
import os

import numpy as np
import pytest

import oracle
from tests.parity import assert_parity

GOLDEN = sorted(p for p in glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz"))
                if os.path.basename(p).startswith(("S0_", "T_", "O_")))


def load(path):
    z = np.load(path, allow_pickle=False)
    return z["rgba"], z["evals"], json.loads(str(z["meta"]))


def test_goldens_present():
    names = {os.path.basename(p)[:-4] for p in GOLDEN}
    assert {"S0_64_P0", "T_64_P0", "O_64_P0"} <= names
    assert len(GOLDEN) >= 9


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p)[:-4] for p in GOLDEN])
def test_oracle_matches_reference_glsl(path):
    rgba, evals, m = load(path)
    img, ev = oracle.render(m["scene"], m["W"], m["H"], pos=m["pos"], mouse=m["mouse"], time=m["time"],
                            max_steps=m["max_steps"])
    assert img.shape == rgba.shape
    s = assert_parity(m["scene"], img, rgba, label=os.path.basename(path))
    # the step counts (sceneSDF calls per pixel) of the reference GLSL run
    assert np.mean(ev == evals) >= 0.99, s
    assert abs(float(ev.mean()) - float(evals.mean())) / float(evals.mean()) < 2e-3
    # alpha is 1 everywhere (gl_FragColor = vec4(col, 1.0))
    assert np.all(img[..., 3] == 1.0)
