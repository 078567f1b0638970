"""cli23 (the joint model's sample driver, src/trigenic_fromtesttrain_2+3.py) against the
reference's own run of that loop (tests/golden/joint/cli/driver.json, written by
tests/golden/make_joint_golden.py), on the CPU: the joint Model runs on the C oracle's engine
(bit-exact with the reference), so stdout and every output file must be byte-identical."""
import json
import os

import pytest

from golden_util import JOINT
from oracle_engine import OracleJointEngine
from trigenicinteractionpredictor_amd import cli23, joint

with open(os.path.join(JOINT, "cli", "driver.json"), encoding="utf-8") as f:
    DRIVER = json.load(f)


@pytest.mark.parametrize("name", sorted(DRIVER))
def test_driver_matches_reference_run_bytewise(name, tmp_path, monkeypatch, capsys):
    run = DRIVER[name]
    monkeypatch.setattr(joint.Model, "Engine", OracleJointEngine)
    d = os.path.join(JOINT, "tiny")
    argv = run["argv"][:5] + [os.path.join(d, "train.dat"), os.path.join(d, "test.dat"),
                              str(run["argv"][5]), str(run["argv"][6])]
    monkeypatch.chdir(tmp_path)
    cli23.main(argv)
    assert capsys.readouterr().out == run["stdout"]
    got = {f: open(f, encoding="utf-8").read() for f in sorted(os.listdir("."))}
    assert sorted(got) == sorted(run["files"])
    for f in got:
        assert got[f] == run["files"][f], f


def test_missing_arguments_take_every_default():
    cfg, _ = cli23.parse(["5", "3"])
    assert cfg == cli23.DEFAULTS
    cfg, seed = cli23.parse(["5", "3", "2", "4", "1", "a", "b", "0", "9"])
    assert cfg == (5, 3, 2, 4, 1, "a", "b", 0) and seed == 9


def test_check_points_follow_the_reference_condition():
    assert cli23.check_points(12, 5) == [0, 5, 10]
    with pytest.raises(ZeroDivisionError):
        cli23.check_points(3, 0)
