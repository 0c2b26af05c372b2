"""The bounds-checked debug build (SURVEY.md §5 "race detection / sanitizers").

``MOPT_KERNEL_CHECKED=1`` loads ``ops/lib/variants/checked`` (compiled with
``-DMOPT_BOUNDS_CHECK``): the kernels verify on the device the data-dependent indices no host
check can see -- token ids, class labels, sorted gather indices -- skip an out-of-range access
instead of faulting, and the host raises ``BoundsViolation`` naming the launch.  Each case runs
in a child process (the library variant is chosen at load time); valid inputs must give
bitwise the default library's results.
"""
import os
import subprocess
import sys
import textwrap

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = {
    "lm": """
        torch.manual_seed(0)
        P, V, d, rpt = 2, 256, 64, 32
        table = torch.randn(P, V, d, device=dev).to(torch.bfloat16).requires_grad_(True)
        tok = torch.randint(0, V, (P * rpt,), device=dev, dtype=torch.int32)
        out = lm.embedding(tok, table, rpt)
        out.float().sum().backward()
        logits = torch.randn(P * rpt, V, device=dev).to(torch.bfloat16)
        labels = torch.randint(0, V, (P * rpt,), device=dev, dtype=torch.int32)
        loss = lm.cross_entropy(logits, labels, rpt)
        res = [out.float().sum().item(), table.grad.float().abs().sum().item(),
               loss.float().sum().item()]
        if BAD:
            tok[5] = V + 3
            try:
                lm.embedding(tok, table, rpt)
                res.append("no error")
            except _lib.BoundsViolation as e:
                res.append("violation: " + str(e)[:80])
        print("RESULT", res)
    """,
    "mlp": """
        from metaopt_amd.models.data import TeacherClassification
        from metaopt_amd.ops.population import MemberConfig, PopulationMLP
        data = TeacherClassification(n_train=256, n_val=128, batch_size=128, seed=0, device=dev)
        pop = PopulationMLP(4, max_width=128, eval_batch=128, device=dev, backend="hip")
        for s, w in enumerate((64, 128)):
            pop.set_member(s, MemberConfig(width=w, lr=0.1, seed=s + 1))
        x, y = data.batch(0)
        pop.train_step(x, y)
        torch.cuda.synchronize()
        res = [float(v) for v in pop.train_loss()[:2]]
        if BAD:
            y = y.clone()
            y[3] = 1000
            try:
                pop.train_step(x, y)
                torch.cuda.synchronize()
                res.append("no error")
            except _lib.BoundsViolation as e:
                res.append("violation: " + str(e)[:80])
        print("RESULT", res)
    """,
}


def _run(case, checked, bad=False):
    code = "import torch\nfrom metaopt_amd.ops import _lib, lm\ndev = torch.device('cuda:0')\n" \
        f"BAD = {bad}\n" + textwrap.dedent(CASES[case])
    env = dict(os.environ, MOPT_KERNEL_CHECKED="1" if checked else "0")
    proc = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True,
                          text=True, timeout=100)
    assert proc.returncode == 0, proc.stderr[-3000:]
    line = [ln for ln in proc.stdout.splitlines() if ln.startswith("RESULT")][-1]
    return eval(line[len("RESULT"):]), proc.stdout


@pytest.mark.parametrize("case", sorted(CASES))
def test_checked_build_matches_default_on_valid_inputs(case):
    plain, _ = _run(case, checked=False)
    checked, _ = _run(case, checked=True)
    # the per-trial loss sums are float atomics (summation order varies run to run)
    assert checked == pytest.approx(plain, rel=1e-5)


@pytest.mark.parametrize("case", sorted(CASES))
def test_checked_build_reports_out_of_range_index(case):
    res, out = _run(case, checked=True, bad=True)
    assert str(res[-1]).startswith("violation"), res
    assert "[mopt bounds]" in out
