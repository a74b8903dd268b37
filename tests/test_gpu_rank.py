"""Rank mode (one process per GPU, RCCL item-block ring, mf_create_rank) rehearsed on the one-GPU
box: two ranks share device 0 and claim distinct RCCL host ids (MFHIP_FAKE_HOSTS), so the ring's
send/recv and the evaluation broadcasts go over loopback sockets.  tools/rank_check.py compares
every rank's factors with an in-process context of the same plan, bit for bit.

The staged path (prepare, run, then rmse / factors with no sync in between, as the JNI
dsgdPrepare / dsgdRun / rmse calls do) with numBlocks = 2 x ranks runs the ring overlap (the last
superstep's second launch on another stream, its send/recv on a third): evaluation has to drain
them before its broadcasts (DSGDforMF.scala:611-619 ring; MatrixFactorization.scala:239-274)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("mode,extra", [
    ("fast", ["--fast-waves", "-8", "--k", "64"]),                       # rank 0 holds no rating
    ("fast", ["--fast-waves", "-8", "--k", "128", "--users", "30000"]),  # both ranks sweep, ring overlap
    ("det", []),
    ("det", ["--users", "30000"])])
def test_rank_mode_staged_eval_matches_single_context(mode, extra):
    env = dict(os.environ, MFHIP_FAKE_HOSTS="1", MFHIP_DEVICE_SHARERS="2", NCCL_DEBUG="WARN",
               MFHIP_TEST="ring_overlap=1")
    port = 29611 + len(extra) + (10 if mode == "det" else 0)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "tools", "rank_check.py"),
           "--mode", mode, "--blocks", "4", "--staged"] + extra
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "RANK_CHECK_OK" in out, out[-3000:]
