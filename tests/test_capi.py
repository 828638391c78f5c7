"""C-ABI checks that need no GPU: libdgprf.so loads, exports every entry point include/dgprf.h
declares, the ctypes structs match the C layout (compiled with gcc), and dgprf_plan_init derives
the reference's layer widths (models/dgp.py:74-115)."""
import ctypes
import json
import os
import re
import subprocess

import pytest

from dgprf import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "dgprf.h")


def declared_functions():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dgprf_[a-z_0-9]+)\s*\(", src)))


def test_exports_every_declared_symbol():
    lib = N.lib()
    names = declared_functions()
    assert len(names) >= 18
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(N.SIGNATURES), set(names) ^ set(N.SIGNATURES)
    assert lib.dgprf_abi_version() == N.ABI_VERSION == 10


def test_struct_layout_matches_c(tmp_path):
    structs = {"dgprf_plan_t": N.Plan, "dgprf_chain_t": N.Chain, "dgprf_batch_t": N.Batch,
               "dgprf_step_t": N.Step}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HDR}"', 'int main(void){',
             'printf("{");']
    first = True
    for cname, cls in structs.items():
        for fname, _ in cls._fields_:
            sep = "" if first else ","
            first = False
            lines.append(f'printf("{sep}\\"{cname}.{fname}\\": %zu", offsetof({cname}, {fname}));')
        lines.append(f'printf(",\\"{cname}.sizeof\\": %zu", sizeof({cname}));')
    lines += ['printf("}");', 'return 0;}']
    c = tmp_path / "layout.c"
    c.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-std=c99", "-o", str(exe), str(c)])
    got = json.loads(subprocess.check_output([str(exe)]).decode())
    for cname, cls in structs.items():
        assert got[f"{cname}.sizeof"] == ctypes.sizeof(cls), cname
        for fname, _ in cls._fields_:
            assert got[f"{cname}.{fname}"] == getattr(cls, fname).offset, (cname, fname)


def test_plan_config2():
    p = N.make_plan(8, 1, [N.RBF] * 3, [1024] * 3, [8, 8, 1], False, N.LIK_GAUSSIAN, 200, 1)
    assert list(p.d[:3]) == [8, 8, 8] and list(p.P[:3]) == [2048] * 3
    assert p.w_total == 2048 * 8 * 2 + 2048 and p.omega_total == 3 * 8 * 1024
    assert p.n_row_tiles == 13 and list(p.ns[:3]) == [16] * 3
    assert all(o % 4 == 0 for o in p.w_off[:3]) and p.ws_chain % 4 == 0


def test_plan_input_cat_and_arc():
    p = N.make_plan(13, 1, [N.RBF, N.ARC], [500, 300], [13, 1], True, N.LIK_GAUSSIAN, 200, 2)
    assert list(p.d[:2]) == [13, 26]          # models/dgp.py:78-79
    assert list(p.P[:2]) == [1000, 300]       # models/dgp.py:103,107
    assert p.ws_total == 2 * p.ws_chain


@pytest.mark.parametrize("bad", [
    dict(kinds=[], n_rf=[], n_gp=[]),
    dict(kinds=[0] * 9, n_rf=[8] * 9, n_gp=[2] * 9),
    dict(kinds=[2], n_rf=[8], n_gp=[2]),
    dict(kinds=[0], n_rf=[0], n_gp=[2]),
    dict(kinds=[0], n_rf=[8], n_gp=[65]),
])
def test_plan_rejects_bad_configs(bad):
    with pytest.raises((ValueError, RuntimeError)):
        N.make_plan(4, 1, bad["kinds"], bad["n_rf"], bad["n_gp"], False, 0, 16, 1)


def test_entry_points_validate_before_enqueue():
    lib = N.lib()
    assert lib.dgprf_sghmc_step(None, None, None, None, None) == N.E_ARG
    p = N.Plan()  # not initialised
    assert lib.dgprf_prior_w(ctypes.byref(p), None, None, None) == N.E_PLAN
    assert lib.dgprf_rf_features(7, None, 0, 1, None, 1, None, None, None) == N.E_ARG
    assert lib.dgprf_philox_normal(None, 4, 0, 0, 1, None) == N.E_ARG
    assert lib.dgprf_error_string(N.E_SHAPE) == b"unsupported shape"


def test_row_group_workspace_bounded():
    """gW partials never exceed 16 rows: workspace for B = 65,536 at config 2's shape holds
    16 x w_total gW floats (host-only plan check, runs without a GPU)."""
    from dgprf import _native as N
    for B, rows in ((200, 13), (256, 16), (257, 9), (1024, 16), (8192, 16), (65536, 16)):
        pl = N.make_plan(8, 1, [N.RBF] * 3, [1024] * 3, [8, 8, 1], False, N.LIK_GAUSSIAN, B, 1)
        assert pl.n_gw_rows == rows, (B, pl.n_gw_rows)
        assert pl.n_rt_pad == 16
        assert (pl.rt_per_group > 1) == (B > 256)


def test_fold_out_plan_choice():
    """Which plans fold the output layer (host-only plan derivation): config 2 at B = 200 with 1-3
    chains; not from 4 chains (wider slices, the chip full of chains), not past B = 256 (row-group
    backward), not configs 3 / 5 (recompute costlier than the boundary) nor softmax outputs."""
    from dgprf import _native as N
    RBFk, ARCk = N.RBF, N.ARC
    mk = lambda kinds, R, g, D, B, C=1, lik=N.LIK_GAUSSIAN: N.make_plan(
        D, g[-1], kinds, R, g, False, lik, B, C)
    assert mk([RBFk] * 3, [1024] * 3, [8, 8, 1], 8, 200).fold_out == 1
    assert mk([RBFk] * 3, [1024] * 3, [8, 8, 1], 8, 200, C=3).fold_out == 1
    assert mk([RBFk] * 3, [1024] * 3, [8, 8, 1], 8, 200, C=4).fold_out == 0
    assert mk([RBFk] * 3, [1024] * 3, [8, 8, 1], 8, 1024).fold_out == 0
    assert mk([ARCk] * 3, [2048] * 3, [9, 9, 1], 9, 200).fold_out == 0
    assert mk([RBFk, ARCk, RBFk, ARCk, RBFk], [8192] * 5, [16] * 4 + [1], 16, 200).fold_out == 0
    assert mk([RBFk] * 2, [1024] * 2, [8, 10], 8, 200, lik=N.LIK_SOFTMAX).fold_out == 0


def test_many_chain_plans_take_one_row_group_per_chain():
    """From 16 chains per launch a plan of <= 16 row tiles whose layers span >= 8 slices takes the
    row-group backward with one row group per chain (dgprf_plan_init): one gW partial row per
    parameter (n_gw_rows = 1) instead of one per 16-row tile; fewer chains, or narrow layers, keep
    the per-row-tile backward."""
    from dgprf import _native as N
    mk = lambda C, B=200, n_rf=4096, n_gp=(30, 30, 10): N.make_plan(
        8, 1, [N.RBF] * 3, [n_rf] * 3, list(n_gp), False, N.LIK_GAUSSIAN, B, C)
    for C in (1, 4, 8):
        p = mk(C)
        assert p.rt_per_group == 1 and p.n_gw_rows == 13
    for C in (16, 64):
        p = mk(C)
        assert min(p.ns[:3]) >= 8
        assert p.rt_per_group == 13 and p.n_gw_rows == 1 and p.fold_out == 0
        p = mk(C, n_rf=1024, n_gp=(8, 8, 1))  # 2 slices per layer: per-row-tile backward
        assert max(p.ns[:3]) < 8 and p.rt_per_group == 1 and p.n_gw_rows == 13
    p = mk(64, B=16)  # one row tile: nothing to group
    assert p.rt_per_group == 1 and p.n_gw_rows == 1
    p = mk(64, B=1000)  # > 16 row tiles: the large-batch row groups (<= 16 partial rows)
    assert p.rt_per_group == 4 and p.n_gw_rows == 16
