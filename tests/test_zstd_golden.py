"""zstd 1.5.2 golden frames (tests/golden/make_zstd_golden.py): the fixture inputs regenerate
from the synthetic corpora, and the reference build (oracle/_ref) reproduces every frame and
round-trips it.  CPU only; the GPU decoder is checked against the same frames in
tests/test_gpu_zstd.py."""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle_lib as O
import lzbench_amd as L

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def cases():
    with open(os.path.join(GOLD, "zstd_manifest.json")) as f:
        return json.load(f)["cases"]


def arrays():
    with np.load(os.path.join(GOLD, "zstd_golden.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def corpus(c):
    if c["corpus"] == "zeros":
        d = np.zeros(c["n"], np.uint8)
        d[::4099] = 7
        return d
    return L.datagen(c["corpus"], c["n"], c["seed"])


@pytest.mark.parametrize("case", cases(), ids=lambda c: c["name"])
def test_inputs_regenerate(case):
    assert hashlib.sha256(corpus(case).tobytes()).hexdigest() == case["input_sha256"]


@pytest.mark.parametrize("case", cases(), ids=lambda c: c["name"])
def test_reference_reproduces_frames(case):
    if not O.have_ref():
        pytest.skip("reference build (oracle/_ref) not present")
    A = arrays()
    data = corpus(case)
    packed, cs = O.compress_chunks(data, "zstd", case["chunk"], case["level"])
    assert (cs == A[case["name"] + "/csizes"]).all()
    assert packed.tobytes() == A[case["name"] + "/packed"].tobytes()
    r, out = O.decompress_chunks(packed, cs, len(data), "zstd", case["chunk"])
    assert r == len(data) and (out == data).all()


def test_reference_version():
    if not O.have_ref():
        pytest.skip("reference build (oracle/_ref) not present")
    assert O.ref().ref_zstd_version() == 10502
