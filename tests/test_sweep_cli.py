"""``mopt sweep`` runs the user's experiment definition on the device path: a ``--name~prior``
space parsed with the hunt grammar and validated against the task, algorithms and options
resolved with the reference's precedence (``--config`` file < command line), ``--gpus N``
launching N ranks (gloo on a CPU host), ``--dtype`` for the optimizer state."""
import json
import math
import os
import subprocess
import sys

import pytest

from metaopt_amd.cli import _space_after_options, main
from metaopt_amd.storage.protocol import get_storage

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMMON = ["--task", "logreg", "--population", "4", "--sync-every", "16", "--steps", "4000"]


def _last_json(out):
    return json.loads(out.strip().splitlines()[-1])


def _trials(name):
    st = get_storage()
    exp = st.fetch_experiments({"name": name})[-1]
    return exp, st.fetch_trials(uid=exp["_id"])


def test_user_prior_defines_the_stored_space_and_the_members(capsys):
    name = "sweep-user-space"
    assert main(["--debug", "sweep", "-n", name, *COMMON, "--max-trials", "12",
                 "--lr~loguniform(0.2, 0.3)", "--weight_decay~loguniform(1e-5, 1e-4)"]) == 0
    out = _last_json(capsys.readouterr().out)
    assert out["experiment"]["space"] == {"/lr": "loguniform(0.2, 0.3)",
                                          "/weight_decay": "loguniform(1e-5, 1e-4)"}
    exp, trials = _trials(name)
    assert exp["metadata"]["priors"] == out["experiment"]["space"]
    assert exp["metadata"]["user_args"][0] == "--lr~loguniform(0.2, 0.3)"
    assert len(trials) >= 12
    for t in trials:
        p = t.params_dict
        assert 0.2 <= p["/lr"] <= 0.3 and 1e-5 <= p["/weight_decay"] <= 1e-4


def test_explicit_double_dash_is_accepted(capsys):
    assert main(["--debug", "sweep", "-n", "sweep-dd", *COMMON, "--max-trials", "4", "--",
                 "--lr~loguniform(0.01, 0.02)"]) == 0
    assert _last_json(capsys.readouterr().out)["experiment"]["space"] == {
        "/lr": "loguniform(0.01, 0.02)"}


def test_default_space_is_the_tasks(capsys):
    from metaopt_amd.worker.tasks import get
    assert main(["--debug", "sweep", "-n", "sweep-default", *COMMON, "--max-trials", "4"]) == 0
    assert _last_json(capsys.readouterr().out)["experiment"]["space"] == get("logreg").priors


def test_unknown_dimension_is_refused():
    with pytest.raises(ValueError, match="not hyper-parameters"):
        main(["--debug", "sweep", "-n", "sweep-bad", *COMMON, "--lr~loguniform(0.1, 1)",
              "--layers~uniform(1, 4, discrete=True)"])


def test_missing_required_dimension_is_refused():
    with pytest.raises(ValueError, match="must define"):
        main(["--debug", "sweep", "-n", "sweep-nolr", *COMMON,
              "--weight_decay~loguniform(1e-5, 1e-4)"])


def test_fidelity_must_be_steps():
    with pytest.raises(ValueError, match="fidelity"):
        main(["--debug", "sweep", "-n", "sweep-fid", *COMMON, "--lr~loguniform(0.1, 1)",
              "--momentum~fidelity(1, 4, 2)"])


def test_a_script_is_refused():
    with pytest.raises(ValueError, match="no script"):
        main(["--debug", "sweep", "-n", "sweep-script", *COMMON, "train.py",
              "--lr~loguniform(0.1, 1)"])


def test_config_file_algorithm_is_honoured(tmp_path, capsys):
    cfg = tmp_path / "sweep.yaml"
    cfg.write_text("algorithms:\n  asha:\n    seed: 3\n    repetitions: .inf\nmax_trials: 10\n")
    assert main(["--debug", "sweep", "-n", "sweep-cfg", *COMMON, "-c", str(cfg),
                 "--lr~loguniform(0.05, 0.5)", "--steps~fidelity(16, 64, 2)"]) == 0
    out = _last_json(capsys.readouterr().out)
    assert list(out["experiment"]["algorithms"]) == ["asha"]
    assert out["experiment"]["algorithms"]["asha"]["seed"] == 3
    exp, trials = _trials("sweep-cfg")
    assert exp["max_trials"] == 10
    assert sum(t.status == "completed" for t in trials) >= 10


def test_command_line_overrides_the_file(tmp_path, capsys):
    cfg = tmp_path / "sweep.yaml"
    cfg.write_text("algorithms:\n  asha:\n    seed: 3\nmax_trials: 50\n")
    assert main(["--debug", "sweep", "-n", "sweep-cfg2", *COMMON, "-c", str(cfg), "--algo",
                 "random", "--max-trials", "6", "--lr~loguniform(0.05, 0.5)"]) == 0
    out = _last_json(capsys.readouterr().out)
    assert list(out["experiment"]["algorithms"]) == ["random"]
    exp, _ = _trials("sweep-cfg2")
    assert exp["max_trials"] == 6


def test_width_prior_sizes_the_population_slots():
    from metaopt_amd.worker.tasks import get
    task, pop, _ = get("mlp").build(2, "cpu", 0, priors={
        "/lr": "loguniform(1e-3, 1)", "/width": "loguniform(64, 192, discrete=True)"})
    assert task.max_width == 192 and pop.max_width == 192
    with pytest.raises(ValueError, match="4096"):
        get("mlp").build(2, "cpu", 0, priors={"/lr": "loguniform(1e-3, 1)",
                                              "/width": "uniform(64, 8192, discrete=True)"})


def test_dtype_selects_the_optimizer_state_precision():
    import torch
    from metaopt_amd.models.llama import PopulationLM
    lm = PopulationLM.__new__(PopulationLM)
    assert lm.moment_dtype == torch.bfloat16          # class default
    from metaopt_amd.worker.tasks import get
    _, pop, _ = get("logreg").build(2, "cpu", 0, state_dtype="fp32")
    assert pop.momentum_dtype == "fp32"


def test_prior_arguments_start_the_user_space():
    assert _space_after_options(["sweep", "-n", "x", "--lr~uniform(0, 1)"]) == \
        ["sweep", "-n", "x", "--", "--lr~uniform(0, 1)"]
    assert _space_after_options(["sweep", "--", "--lr~u"]) == ["sweep", "--", "--lr~u"]
    assert _space_after_options(["hunt", "-n", "x", "s.py", "--lr~u"]) == \
        ["hunt", "-n", "x", "s.py", "--lr~u"]
    assert _space_after_options(["-v", "sweep", "--lr~u"]) == ["-v", "sweep", "--", "--lr~u"]


@pytest.mark.parametrize("argv", [
    ["hunt", "-n", "sweep", "./train.py", "--lr~uniform(0,1)"],        # experiment named sweep
    ["hunt", "-n", "x", "./train.py", "--mode", "sweep", "--lr~u"],    # a user value "sweep"
    ["-v", "hunt", "-n", "x", "./sweep", "--lr~u"],
])
def test_sweep_token_outside_the_subcommand_is_left_alone(argv):
    """Only the ``sweep`` sub-command is rewritten: a stray ``--`` in a hunt's user arguments
    would change the CommandLineConflict fingerprint and branch a resumed experiment."""
    assert _space_after_options(argv) == argv


def test_gpus_two_spawns_two_ranks(tmp_path):
    """``--gpus 2`` on a CPU host: two gloo ranks, rank 0 writes the experiment."""
    db = tmp_path / "db.pkl"
    env = dict(os.environ, MOPT_DB_TYPE="pickleddb", MOPT_DB_ADDRESS=str(db),
               ORION_DB_TYPE="pickleddb", ORION_DB_ADDRESS=str(db), OMP_NUM_THREADS="2",
               PYTHONPATH=ROOT)
    env.pop("WORLD_SIZE", None)
    proc = subprocess.run([sys.executable, "-m", "metaopt_amd", "sweep", "-n", "two-ranks",
                           *COMMON, "--gpus", "2", "--max-trials", "16",
                           "--lr~loguniform(0.05, 0.5)"],
                          cwd=str(tmp_path), env=env, capture_output=True, text=True,
                          timeout=300)
    assert proc.returncode == 0, proc.stderr[-3000:]
    out = _last_json(proc.stdout)
    assert out["experiment"]["world_size"] == 2
    assert out["completed"] >= 16 and math.isfinite(out["best_val_loss"])
