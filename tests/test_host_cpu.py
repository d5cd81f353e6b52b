"""Host-side logic that needs no GPU: scenario/config parsing, spawn and
sharding arithmetic, algorithmic byte counts."""
import json
import os
import sys

import numpy as np
import pytest

from lnw.config import Scenario
from lnw import shard

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_scenario_from_reference_config(tmp_path):
    cfg = {"overall": {"discrete": False, "landing_ops": True, "tactics": "aggressive"},
           "environment_setup": {"ew_threshold": 70, "movement_threshold": 74, "side": "blue",
                                 "n_blue": 3, "n_red": 2, "n_red_landingship": 1,
                                 "red_aggression": 0.4, "trained_red": True},
           "hyperparameters": {"episode_steps": 40}}
    p = tmp_path / "config.json"
    p.write_text(json.dumps(cfg))
    s = Scenario.from_config(str(p))
    P = s.params()
    assert (P.discrete, P.landing_ops, P.aggressive, P.side_blue, P.trained_red) == (0, 1, 1, 1, 1)
    assert (P.move_thr, P.ew_thr, P.lz_x, P.lz_y) == (74, 70, 14, 82)
    assert P.red_aggression == 0.4 and s.n_red_landingship == 1
    s2 = Scenario.from_config(str(p), tactics="defensive", side="red")
    assert s2.params().aggressive == 0 and s2.params().side_blue == 0


def test_shard_partition_covers_all_envs():
    for total in (1, 7, 64, 65536, 65537):
        for world in (1, 2, 3, 8):
            spans = [shard.env_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def test_algorithmic_bytes():
    sys.path.insert(0, ROOT)
    import bench
    # 4v4: actions 128 + obs 2176 + rewards/done/cog 40 + state 2*(8*26+52)
    assert bench.algorithmic_bytes(4, 4) == 128 + 2176 + 40 + 2 * (8 * 26 + 52)
    # quiet steps write back cell, radar and step counter per agent and the env's step counter
    assert bench.algorithmic_bytes(4, 4, quiet=True) == 128 + 2176 + 40 + (8 * 26 + 52) + (8 * 12 + 4)


def test_packaged_grid_is_the_reference_grid():
    from lnw.batched import default_grid
    g = np.load(os.path.join(ROOT, "tests", "golden", "grids.npz"))
    assert np.array_equal(default_grid(100), g["grid100"])
    assert np.array_equal(default_grid(200), g["grid200"])


def test_measured_traffic_keyed_to_sources(tmp_path, monkeypatch):
    """bench.py reports roofline.traffic only for the in-tree library built from
    the sources profiles/traffic.json was measured on (lnw.build.source_digest):
    a different digest, or another library through LNW_LIB, gives null."""
    sys.path.insert(0, ROOT)
    import bench
    from lnw import build

    class Args:
        workload, spawns, los_mode, move_mode = "reference", "reference", 0, 0

    prof = tmp_path / "profiles"
    prof.mkdir()
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.delenv("LNW_LIB", raising=False)
    key = "reference_e64_los0_mv0"
    tj = {"src_sha256": build.source_digest(), "launch_bytes": {key: 123.0}}
    (prof / "traffic.json").write_text(json.dumps(tj))
    fresh = os.path.exists(build.OUT) and all(
        os.path.getmtime(d) <= os.path.getmtime(build.OUT) for d in build.DEPS)
    assert bench.measured_traffic(Args, 64) == (123.0 if fresh else None)
    assert bench.measured_traffic(Args, 128) is None  # no record for this workload
    monkeypatch.setenv("LNW_LIB", str(tmp_path / "other.so"))
    assert bench.measured_traffic(Args, 64) is None
    monkeypatch.delenv("LNW_LIB")
    tj["src_sha256"] = "0" * 64
    (prof / "traffic.json").write_text(json.dumps(tj))
    assert bench.measured_traffic(Args, 64) is None


def test_source_digest_ignores_tree_location(monkeypatch):
    """The digest hashes flags without include paths and file contents by
    basename, so the GPU box (another tree path) computes the same value."""
    from lnw import build
    d = build.source_digest()
    assert len(d) == 64
    monkeypatch.setattr(build, "INCLUDE", "/elsewhere/include")
    monkeypatch.setattr(build, "CSRC", "/elsewhere/csrc")
    assert "-I/elsewhere/include" in build.flags()
    assert build.source_digest() == d
