"""Time/arrival-range sharding of one non-keyed stream: 2 ranks (one process each, both on
cuda:0, exchange over gloo with host staging -- the protocol is identical to RCCL device all-gathers) must
produce exactly the windows the single-stream oracle produces, out-of-order tuples across chunk boundaries
included; cases 4-5 are count windows (the count path's per-rank count cells, BASELINE configs[4]), cases 6-7
count + time windows on the count path (scotty_shard_push_timed)."""
import json
import os
import subprocess
import sys

import pytest

from helpers import build_ops, same_windows, ROOT
from shard_cases import case
from oracle.oracle import JavaError

pytestmark = pytest.mark.gpu


def _run_sharded(tmp_path, cid, nproc, backend, sync=False):
    out = str(tmp_path / "w.json")
    port = str(29500 + cid + 8 * nproc + (os.getpid() % 400) + (1000 if sync else 0))
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", SCOTTY_SHARD_SYNC="1" if sync else "0")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
                        "--master-addr", "127.0.0.1", "--master-port", port,
                        os.path.join(ROOT, "tests", "shard_worker.py"), out, str(cid), backend],
                       env=env, capture_output=True, text=True, timeout=240)
    return r, out


@pytest.mark.parametrize("cid,sync", [(0, False), (1, False), (4, False), (6, False), (7, False), (0, True), (6, True)])
def test_rccl_exchange_single_rank_matches_oracle(tmp_path, cid, sync):
    """The RCCL ("nccl") exchange path on one rank of this one-GPU box: time windows (in order and out of order),
    count windows, count + time windows; the exchange buffer is poisoned on torch's stream before every chunk.
    Default: the all-gather queued on the op's own stream between the push and the commit (no host
    synchronisation; the worker records that this mode ran); sync: SCOTTY_SHARD_SYNC=1, the push and torch's stream
    synchronised by the host on both sides."""
    r, out = _run_sharded(tmp_path, cid, 1, "nccl", sync)
    _check(r, out, cid, 1)
    assert open(out + ".rank0.mode").read() == ("sync" if sync else "async")


@pytest.mark.parametrize("cid", [0, 1, 2, 3, 4, 5, 6, 7])
def test_two_rank_sharded_stream_matches_oracle(tmp_path, cid):
    r, out = _run_sharded(tmp_path, cid, 2, "gloo")
    _check(r, out, cid, 2)


def _check(r, out, cid, nproc):
    tb = r.stderr.find("Traceback")
    assert r.returncode == 0, r.stderr[tb:tb + 3000] if tb >= 0 else r.stderr[-3000:]
    outs = [json.load(open("%s.rank%d" % (out, k))) for k in range(nproc)]
    for k in range(1, nproc):  # every rank emits the same rows (replicated slice store)
        assert outs[k] == outs[0], ("rank %d differs from rank 0" % k)
    got = outs[0]
    cfg, ts, vals, sched = case(cid)
    _, ora = build_ops(cfg)
    k = 0
    fails = 0
    for st in sched:
        if st[0] == "push":
            fails += ora.processElements(ts[st[1]:st[2]], vals[st[1]:st[2]])
        else:
            g = got[k]
            k += 1
            if g == [["index_error"]]:
                with pytest.raises(JavaError):
                    ora.processWatermark(st[1])
                continue
            exp = ora.processWatermark(st[1])
            assert g[-1] == ["dropped", fails]
            rows = g[:-1]
            assert len(rows) == len(exp), (len(rows), len(exp))
            for x, y in zip(rows, exp):
                assert (x[0], x[1], x[2], bool(x[3])) == (y.getStart(), y.getEnd(), y.getMeasure(), y.hasValue()), (x, y)
                assert x[4] == y.getAggValues(), (x, y)
    assert k > 0
