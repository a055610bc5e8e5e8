"""The mapper's BA half on CPU: the config / driver contract and the oracle-stage pipeline (oracle/mapper.py) that
the GPU mapper test checks against (global_mapper.py:80-146)."""
import contextlib
import io

import numpy as np
import pytest

import mapper_scene as MS
from instantsfm_amd.controllers.config import GENERAL_OPTIONS, OUT_OF_SCOPE_STAGES, Config
from instantsfm_amd.controllers.global_mapper import SolveGlobalMapper
from instantsfm_amd.synth import write_mapper_database


def _similarity_residual(C, G):
    """Max distance after the best similarity mapping C onto G (camera centres are fixed up to a similarity)."""
    mc, mg = C.mean(0), G.mean(0)
    U, sv, Vt = np.linalg.svd((G - mg).T @ (C - mc))
    R = U @ Vt
    s = sv.sum() / np.sum((C - mc) ** 2)
    return np.linalg.norm(s * (C - mc) @ R.T + mg - G, axis=1).max()


def test_config_matches_reference_defaults():
    cfg = Config('colmap')
    assert cfg.OPTIONS == GENERAL_OPTIONS
    assert cfg.BUNDLE_ADJUSTER_OPTIONS['function_tolerance'] == 5e-4
    assert cfg.INLIER_THRESHOLD_OPTIONS['max_reprojection_error'] == 1e-2
    assert cfg.TRIANGULATOR_OPTIONS['ba_global_max_refinements'] == 5
    with pytest.raises(ValueError):
        Config('superpoint')
    half = Config.for_ba_half()
    assert all(half.OPTIONS[k] for k in OUT_OF_SCOPE_STAGES) and not half.OPTIONS['skip_retriangulation']
    assert not GENERAL_OPTIONS['skip_preprocessing']  # the module default is untouched


@pytest.mark.parametrize("stage", OUT_OF_SCOPE_STAGES)
def test_mapper_refuses_out_of_scope_stages(stage):
    cfg = Config.for_ba_half()
    cfg.OPTIONS[stage] = False
    with pytest.raises(NotImplementedError):
        SolveGlobalMapper(None, [], [], cfg)


def test_mapper_database_contents(tmp_path):
    scene = MS.make_db(tmp_path / "db.db")
    vg, cams, ims, cfg = MS.load(tmp_path / "db.db", scene)
    assert len(ims) == 40 and len(cams) == 4 and len(vg.image_pairs) == scene.n_pairs
    assert sum(len(p.matches) for p in vg.image_pairs.values()) == scene.n_matches
    assert all(im.is_registered for im in ims)
    assert all(np.asarray(im.features).dtype == np.float32 for im in ims)
    # rotations: GT composed with a 0.1 deg perturbation
    ang = [np.degrees(np.arccos(np.clip((np.trace(im.world2cam[:3, :3] @ R.T) - 1) / 2, -1, 1)))
           for im, R in zip(ims, scene.rot_gt)]
    assert 0 < max(ang) < 0.6


def test_oracle_mapper_recovers_geometry(tmp_path):
    """The oracle pipeline, from random GP positions, reaches the noise floor and the ground-truth camera centres up
    to a similarity: the checker itself is sound."""
    from oracle import mapper as OM
    scene = MS.make_db(tmp_path / "db.db")
    vg, cams, ims, cfg = MS.load(tmp_path / "db.db", scene)
    np.random.seed(0)
    trace = []
    with contextlib.redirect_stdout(io.StringIO()):
        OM.solve_global_mapper(vg, cams, ims, cfg, trace=trace)
    names = [t[0] for t in trace]
    assert names == ['tracks', 'gp', 'gp_filtered', 'ba0', 'ba1', 'ba2', 'ba_filtered', 'ba_final', 'retri_filtered']
    final_rmse = dict((t[0], t[3]) for t in trace)['ba_final']
    assert 0.4 < final_rmse < 0.8, final_rmse  # 0.5 px observation noise, outliers filtered
    C = np.array([im.center() for im in ims])
    assert _similarity_residual(C, scene.centers_gt) < 0.3  # ring radius 30
    # most of the tracks survive (1 % outliers, 1 % wrong matches)
    assert trace[-1][1] > 0.95 * trace[0][1]
