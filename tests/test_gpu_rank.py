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


def run_ranks(cmd, env, timeout):
    """The launcher and its ranks in a process group of their own: on a timeout the whole group is
    killed, so no rank is left holding the device."""
    import signal
    p = subprocess.Popen(cmd, env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                         start_new_session=True)
    try:
        out, _ = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        out, _ = p.communicate()
        return -9, (out or "") + "\n[timeout]"
    return p.returncode, out


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
    rc, out = run_ranks(cmd, env, 240)
    assert rc == 0 and "RANK_CHECK_OK" in out, out[-3000:]


@pytest.mark.parametrize("mode,extra", [
    ("det", []),                            # bitwise against one context: the reference order is plan-free
    ("fast", ["--fast-waves", "-16"])])     # uniform G: bitwise against 8 in-process virtual shards
def test_rank_mode_yahoo_shaped_world8(mode, extra):
    """BASELINE config 4 (Yahoo-Music-shaped, k = 256, numBlocks = 8, "on 8 x MI355X") through the
    rank path at 0.05 scale (91k users x 6.8k items x 36M ratings): 8 ranks share device 0, each
    owning one user block, the item blocks rotating over the RCCL ring (DSGDforMF.scala:262-357,
    611-619).  One epoch; factors compared bit for bit (tools/rank_check.py).  The fast case is
    the one that caught the k = 256 lean-path defect (profiles/r04_k256_repeatability.txt)."""
    env = dict(os.environ, MFHIP_FAKE_HOSTS="1", MFHIP_DEVICE_SHARERS="8", NCCL_DEBUG="WARN")
    port = 29661 + (10 if mode == "det" else 0)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "tools", "rank_check.py"),
           "--mode", mode, "--config", "YAHOO", "--scale", "0.05", "--iterations", "1"] + extra
    rc, out = run_ranks(cmd, env, 280)
    assert rc == 0 and "RANK_CHECK_OK" in out, out[-3000:]
