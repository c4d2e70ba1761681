"""The zstd decoder's counted-wait invariant, checked on the built code object (CPU only).

`lzh_zstd_seq_kernel` and `lzh_zstd_huf{,8}_kernel` (lzbench_amd/csrc/decode_hip.hip) wait at each
uniform point with `s_waitcnt vmcnt(16)` and rely on the 16 steps of the interval before it issuing at
least 16 vector-memory operations after the previous point's LDS-DMA fills (one record / byte store
per step, a dummy one when a lane has none).  tools/vmcnt_check.py walks every path of the disassembled
kernels; these tests run it on the object the library is linked from, and show that it catches the
defects that would break the invariant (a step without its store, a shorter interval).  An EXTRA
vector-memory operation only makes the wait stricter, so it is accepted.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import vmcnt_check as V  # noqa: E402

OBJ = os.path.join(ROOT, "build", "obj", "decode_hip.o")
pytestmark = pytest.mark.skipif(not os.path.exists(f"{V.LLVM}/llvm-objdump"), reason="no ROCm llvm tools")


@pytest.fixture(scope="module")
def dis():
    if not os.path.exists(OBJ):
        subprocess.run(["make", "-C", os.path.join(ROOT, "lzbench_amd", "csrc"), "-j8"], check=True)
    return V.disassemble(OBJ)


@pytest.mark.parametrize("kernel", V.KERNELS)
def test_invariant_holds_at_head(dis, kernel):
    assert V.check_listing(V.kernel_listing(dis, kernel), kernel) == []


def _step_stores(lst):
    """indices of the per-step stores: stores of the block that ends in the counted loop's back edge"""
    out = []
    for i, (_, ins) in enumerate(lst):
        if ins.startswith(("global_store", "buffer_store")):
            tail = [x for _, x in lst[i:i + 6]]
            if any(t.startswith(("s_cbranch_scc0", "s_cbranch_scc1")) for t in tail):
                out.append(i)
    return out


@pytest.mark.parametrize("kernel", V.KERNELS)
def test_missing_step_store_is_caught(dis, kernel):
    lst = V.kernel_listing(dis, kernel)
    idx = _step_stores(lst)
    assert idx, "no per-step store found next to the step loop's back edge"
    bad = list(lst)
    bad[idx[-1]] = (bad[idx[-1]][0], "s_nop 0")          # one store of the unrolled step gone
    assert V.check_listing(bad, kernel, base=lst[0][0]), "a step without its store must be reported"


@pytest.mark.parametrize("kernel", V.KERNELS)
def test_short_interval_is_caught(dis, kernel):
    lst = V.kernel_listing(dis, kernel)
    inits = [i for i, (_, ins) in enumerate(lst) if ins.replace(",", " ").split()[:1] == ["s_mov_b32"]
             and ins.replace(",", " ").split()[-1] == "16"]
    assert inits, "no step-loop counter initialised to 16"
    bad = list(lst)
    for i in inits:
        a, ins = bad[i]
        bad[i] = (a, ins[:ins.rindex("16")] + "14")         # 14 steps between the points
    assert V.check_listing(bad, kernel, base=lst[0][0]), "an interval of 14 steps must be reported"


def test_extra_operation_is_safe(dis):
    kernel = "lzh_zstd_seq_kernel"
    lst = V.kernel_listing(dis, kernel)
    idx = _step_stores(lst)
    bad = list(lst)
    # a vector ALU instruction of the step turned into one more load (a scalar one may be the loop
    # counter's compare, which the checker's constant tracking needs)
    j = max(i for i in range(idx[0]) if bad[i][1].startswith("v_"))
    a, ins = bad[j]
    bad[j] = (a, "global_load_dword v0, v[0:1], off")
    assert V.check_listing(bad, kernel, base=lst[0][0]) == []
