"""Row-sharded mode (sharded.py) on the GPU: world 1 in-process against KGAT, and world 2
(two ranks on the one test GPU, gloo host-staged) through tests/sharded_worker.py."""
from __future__ import annotations

import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist

from tests.conftest import ROOT, load_pkg

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def pkg():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return load_pkg()


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_logged(cmd, env, log_name: str, timeout: int):
    """Run a multi-rank command with its stdout / stderr streamed into gpurun_out/<log_name> as it runs (the
    ranks' progress lines show up there), then read it back: (returncode, stdout, stderr)."""
    out = ROOT / "gpurun_out"
    out.mkdir(exist_ok=True)
    fo, fe = out / f"{log_name}.out", out / f"{log_name}.err"
    with open(fo, "w") as so, open(fe, "w") as se:
        rc = subprocess.run(cmd, cwd=ROOT, env=env, stdout=so, stderr=se, text=True, timeout=timeout).returncode
    return subprocess.CompletedProcess(cmd, rc, fo.read_text(), fe.read_text())


def test_sharded_world1_matches_kgat(pkg):
    graph = __import__(pkg.__name__ + ".graph", fromlist=["graph"])
    sh = __import__(pkg.__name__ + ".sharded", fromlist=["sharded"])
    if not dist.is_initialized():
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    U, E, inter, trip = graph.synthetic_ckg(8000, 60000, seed=9)
    lay = graph.build_layout(U, E, inter, trip)
    args = pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(lay.rel_order), layer_size=[64, 32, 16],
                        message_dropout=[0.0, 0.0, 0.0])
    torch.manual_seed(3)
    ref = pkg.KGAT(args)
    ref.attach_graph(lay, DEV)
    m = sh.RowShardedKGAT(args, lay, sh.Comm(), DEV)
    m.load_full_state(ref.state_dict())
    rng = np.random.default_rng(1)
    n_items = int(inter[:, 1].max()) + 1
    b = [torch.from_numpy(x).to(DEV) for x in (rng.integers(0, U, 128), rng.integers(0, n_items, 128),
                                                  rng.integers(0, n_items, 128))]
    lr = ref(*b, mode=pkg.KGATMode.TRAIN_CF)
    lr.backward()
    ls = m(*b, mode=pkg.KGATMode.TRAIN_CF)
    ls.backward()
    assert abs(ls.item() - lr.item()) < 1e-6
    np.testing.assert_allclose(m._user_entity_embedding_shard.grad.cpu().numpy(),
                               ref._user_entity_embedding.weight.grad.cpu().numpy(), atol=1e-6, rtol=1e-4)
    for a, w in zip(m._cf_weights(), ref._cf_weights()):
        np.testing.assert_allclose(a.grad.cpu().numpy(), w.grad.cpu().numpy(), atol=1e-5, rtol=1e-4)
    ref.build_optimizer(1e-3, 1e-4)
    m.build_optimizer(1e-3, 1e-4)
    ref.update_cf_weights()
    m.update_cf_weights()
    np.testing.assert_allclose(m._user_entity_embedding_shard.detach().cpu().numpy(),
                               ref._user_entity_embedding.weight.detach().cpu().numpy(), atol=2e-5)
    # KG step on the same batch
    kg = [torch.from_numpy(x).to(DEV) for x in (rng.integers(0, U + E, 64), rng.integers(0, len(lay.rel_order), 64),
                                                   rng.integers(0, U + E, 64), rng.integers(0, U + E, 64))]
    lr = ref(*kg, mode=pkg.KGATMode.TRAIN_KG)
    lr.backward()
    ls = m(*kg, mode=pkg.KGATMode.TRAIN_KG)
    ls.backward()
    assert abs(ls.item() - lr.item()) < 1e-6
    np.testing.assert_allclose(m._user_entity_embedding_shard.grad.cpu().numpy(),
                               ref._user_entity_embedding.weight.grad.cpu().numpy(), atol=1e-6, rtol=1e-4)
    np.testing.assert_allclose(m._trans_matrix.grad.cpu().numpy(), ref._trans_matrix.grad.cpu().numpy(), atol=1e-6,
                               rtol=1e-4)
    ref.eval()
    m.eval()
    att = [torch.from_numpy(x).to(DEV) for x in (lay.heads, lay.rels, lay.tails)] + [torch.tensor(lay.rel_order)]
    ref(*att, mode=pkg.KGATMode.UPDATE_ATTENTION)
    m(*att, mode=pkg.KGATMode.UPDATE_ATTENTION)
    np.testing.assert_allclose(m.shard.local_val.cpu().numpy(), ref.graph().A.val.cpu().numpy(), rtol=1e-4,
                               atol=1e-6)
    tabs_s, tabs_r = m.propagate(), ref.propagate()
    for a, w in zip(tabs_s, tabs_r):
        np.testing.assert_allclose(a.cpu().numpy(), w.cpu().numpy(), atol=1e-5, rtol=1e-4)
    users, items = torch.arange(40, device=DEV), torch.arange(200, device=DEV)
    with torch.no_grad():
        np.testing.assert_allclose(m(users, items, mode=pkg.KGATMode.PREDICT).cpu().numpy(),
                                   ref(users, items, mode=pkg.KGATMode.PREDICT).cpu().numpy(), atol=1e-5, rtol=1e-4)


@pytest.mark.parametrize("fuse", [False, True])
def test_bad_gathered_hop_id_raises_index_error(pkg, fuse):
    """the hop backward's all-peer gather hands a rank row ids no local code produced (the
    round-5 fault: uninitialised peer blocks used as rows).  With one gathered id out of range the step
    does not fault: kgat_map_build_checked drops it, update_cf_weights raises IndexError with no parameter
    or Adam moment moved and the deferred table update dropped, and the next good step equals a fresh
    model's same step bit for bit.  (World 1 over gloo with the transport forced on: the rank's own block
    of the gathered id list is corrupted in flight, as a peer's would be.)"""
    graph = __import__(pkg.__name__ + ".graph", fromlist=["graph"])
    sh = __import__(pkg.__name__ + ".sharded", fromlist=["sharded"])
    if not dist.is_initialized():
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)

    class CorruptIds(sh.Comm):
        corrupted = 0

        def gather_at(self, send, out, starts, sizes):
            pend = super().gather_at(send, out, starts, sizes)
            if out.dtype == torch.int32 and out.dim() == 1 and self.arm and int(sizes[0]) > 3:
                out[3] = 1 << 30  # a peer's corrupt row id
                CorruptIds.corrupted += 1
            return pend

    U, E, inter, trip = graph.synthetic_ckg(8000, 60000, seed=9)
    lay = graph.build_layout(U, E, inter, trip)
    args = pkg.KGATArgs(user_num=U, entity_num=E, relation_num=len(lay.rel_order), layer_size=[64, 32],
                        message_dropout=[0.0, 0.0])
    torch.manual_seed(3)
    ref = pkg.KGAT(args)
    models = []
    for arm in (True, False):
        comm = CorruptIds(force=True)
        comm.arm = arm
        m = sh.RowShardedKGAT(args, lay, comm, DEV)
        m.load_full_state(ref.state_dict())
        m.build_optimizer(1e-3, 1e-4)
        m.fuse_table_update = fuse
        models.append(m)
    bad, good = models
    rng = np.random.default_rng(1)
    n_items = int(inter[:, 1].max()) + 1
    b = [torch.from_numpy(x).to(DEV) for x in (rng.integers(0, U, 128), rng.integers(0, n_items, 128),
                                                  rng.integers(0, n_items, 128))]
    before = {k: v.detach().clone() for k, v in bad.state_dict().items() if not v.is_sparse}
    bad(*b, mode=pkg.KGATMode.TRAIN_CF).backward()
    assert CorruptIds.corrupted >= 1  # the hop layer's gathered id list went through the corrupting gather
    with pytest.raises(IndexError):
        bad.update_cf_weights()
    after = {k: v.detach() for k, v in bad.state_dict().items() if not v.is_sparse}
    assert all(torch.equal(before[k], after[k]) for k in before)
    assert not bad._cf_optimizer.state and bad._table_update.pending is None
    assert all(p.grad is None for p in bad.parameters())
    # the next (good) step: the same bits as a model that never saw the bad one
    bad.comm.arm = False
    for m in models:
        m(*b, mode=pkg.KGATMode.TRAIN_CF).backward()
        m.update_cf_weights()
    for (k, pa), (_, pb) in zip(bad.named_parameters(), good.named_parameters()):
        if not pa.is_sparse:
            assert torch.equal(pa, pb), k


@pytest.mark.parametrize("world,dims,chunk", [(2, "64:64,32", 0), (2, "256:256,128,64", 0), (4, "256:256,128,64", 0),
                                              (3, "256:256,128,64", 64), (8, "256:256,128,64", 0),
                                              (8, "64:64,32", 0)])
def test_sharded_ranks_one_gpu(world, dims, chunk):
    """tests/sharded_worker.py on `world` ranks sharing this GPU (gloo, host-staged): the row-sharded
    model vs single-GPU KGAT on the global batch -- at the C2 shape and at C5's (d = 256, layers
    [256, 128, 64], configs[4]) -- CF and KG loss, gradient shards, Adam, attention refresh, PREDICT.
    With the whole-width gather (chunk 0, the default) the propagated tables, the refreshed values
    and the table gradients are the single GPU's bit for bit (same rows, same edges, same order);
    64-column chunks (KGAT_SHARD_CHUNK) change the hub rows' summation order: tolerance only."""
    env = dict(os.environ, SHARDED_WORKER_DIMS=dims, KGAT_SHARD_CHUNK=str(chunk))
    env["PYTHONPATH"] = str(ROOT) + os.pathsep + env.get("PYTHONPATH", "")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(ROOT / "tests" / "sharded_worker.py")]
    p = _run_logged(cmd, env, f"sharded_world{world}_d{dims.split(':')[0]}_c{chunk}", timeout=600)
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
    assert p.stdout.count("sharded parity ok") == world, p.stdout[-2000:]
    if chunk == 0:
        import re
        flags = re.findall(r"bit-identical (\{[^}]*\})", p.stdout)  # rank lines may interleave
        assert len(flags) == world and all("False" not in f for f in flags), flags


def test_dp_sharded_grad_sync_world2_matches_allreduce():
    """replicas.ShardedGradSync (row-block exchange, owned-row Adam, all-gather) vs all-reduce + full
    Adam over 3 CF steps on two ranks (tests/dp_worker.py): bit-identical parameters, identical replicas."""
    env = dict(os.environ)
    env["PYTHONPATH"] = str(ROOT) + os.pathsep + env.get("PYTHONPATH", "")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(ROOT / "tests" / "dp_worker.py")]
    p = _run_logged(cmd, env, "dp_world2", timeout=600)
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])


def test_dp_exchange_paths_world4():
    """tests/dp_worker.py on four ranks (all on this GPU, gloo): every exchange path (all-reduce,
    row-block reduce-scatter with and without the backward overlap, replicated hop-set exchange,
    its dense fallback with rank 1 dense, the fused table update) keeps the replicas identical, and
    the fused replicated path equals the unfused one bit for bit -- the union / merge over G = 4
    lists the 8-GPU run takes, minus RCCL."""
    env = dict(os.environ)
    env["PYTHONPATH"] = str(ROOT) + os.pathsep + env.get("PYTHONPATH", "")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=4",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(ROOT / "tests" / "dp_worker.py")]
    p = _run_logged(cmd, env, "dp_world4", timeout=600)
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])


def test_dp_replicated_exchange_wide_layer0_world2():
    """a 128-wide layer 0 (128 -> 128, no fused saved-state backward) under
    ShardedGradSync(replicate_table=True): each rank's compact hop buffers hold exactly its own
    (different) hop count, so the hop-set all-gather must pad to the largest; paths A-E as in
    tests/dp_worker.py, with d = 128 and layers [128, 64]."""
    env = dict(os.environ)
    env["PYTHONPATH"] = str(ROOT) + os.pathsep + env.get("PYTHONPATH", "")
    env["DP_WORKER_DIMS"] = "128:128,64"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(ROOT / "tests" / "dp_worker.py")]
    p = _run_logged(cmd, env, "dp_world2_wide", timeout=600)
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])


@pytest.mark.parametrize("world", [2, 4, 8])
def test_dp_exchange_paths_c4_shape(world):
    """C4's exact shape (d = 128, layers [128, 64, 32], configs[3]) through every
    data-parallel exchange path of tests/dp_worker.py on `world` ranks sharing this GPU (gloo) -- the
    3-layer sharded table exchange bench.py runs for C4 (row-block reduce-scatter, owned-row Adam,
    all-gather), with and without the backward overlap (attach), and with frontier_forward + the fused
    table update on (path H, bit-identical to C); replicas identical on every path, B / C bit-equal to
    the all-reduce path A at world 2."""
    env = dict(os.environ, DP_WORKER_DIMS="128:128,64,32")
    env["PYTHONPATH"] = str(ROOT) + os.pathsep + env.get("PYTHONPATH", "")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(ROOT / "tests" / "dp_worker.py")]
    p = _run_logged(cmd, env, f"dp_world{world}_c4shape", timeout=600)
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
    assert p.stdout.count(": OK") == world, p.stdout[-2000:]


def test_ddp_wrapped_kgat_gradients_are_rank_means():
    """KGAT inside torch.nn.parallel.DistributedDataParallel (gloo, two ranks on this GPU,
    tests/ddp_worker.py): with the direct backward off (its default) a plain ``loss.backward()`` goes through
    the autograd engine, DDP's reducer runs, and the table / aggregator gradients are the mean over ranks."""
    env = dict(os.environ)
    env["PYTHONPATH"] = str(ROOT) + os.pathsep + env.get("PYTHONPATH", "")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(ROOT / "tests" / "ddp_worker.py")]
    p = _run_logged(cmd, env, "ddp_world2", timeout=300)
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
    assert p.stdout.count("DDP OK") == 2, p.stdout[-2000:]


def test_rccl_world1_collectives_match_gloo():
    """every collective of replicas.py / sharded.py through RCCL (backend "nccl",
    world 1 on the box's GPU, forced) vs the gloo / no-exchange paths (tests/rccl_worker.py)."""
    env = dict(os.environ)
    env["PYTHONPATH"] = str(ROOT) + os.pathsep + env.get("PYTHONPATH", "")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(ROOT / "tests" / "rccl_worker.py")]
    p = _run_logged(cmd, env, "rccl_world1", timeout=600)
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
    assert "rccl world1: OK" in p.stdout, p.stdout[-2000:]


@pytest.mark.parametrize("dp,gpus,config,scale", [("replicated", 2, "small", 0.2), ("sharded", 2, "small", 0.2),
                                                  ("replicated", 4, "small", 0.2), ("sharded", 2, "c4", 0.01),
                                                  ("replicated", 8, "c2", 0.02), ("sharded", 8, "c4", 0.002)])
def test_bench_two_ranks_gloo_rehearsal(dp, gpus, config, scale):
    """bench.py --gpus 2 end to end (launch, process group, DP replicas with the table exchange, timing,
    max-over-ranks, one JSON line) with both ranks on this one GPU over gloo (KGAT_BENCH_BACKEND):
    the N-rank path the driver's multi-GPU run takes, minus RCCL -- also at C4's shape (d = 128,
    [128, 64, 32], 1 % scale) with the sharded exchange and its frontier leg."""
    import json
    import subprocess
    import sys

    env = dict(os.environ, KGAT_BENCH_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = _run_logged([sys.executable, str(ROOT / "bench.py"), "--gpus", str(gpus), "--config", config, "--scale",
                     str(scale), "--steps", "3", "--warmup", "1", "--dp", dp], env, f"bench_{dp}_{gpus}_{config}",
                    timeout=400)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == gpus and rec["config"]["parallelism"] == f"dp{gpus}" and rec["config"]["dp_exchange"] == dp
    assert rec["rehearsal"].startswith("gloo") and rec["value"] > 0 and np.isfinite(rec["final_loss"])
    assert sum(rec["dp_table_exchange_steps"].values()) == 4 if dp == "replicated" else True
    fr = rec["frontier_forward"]  # the frontier-forward leg (composes with either exchange) ran too
    assert fr["bpr_pairs_per_s"] > 0
    if dp == "replicated":
        assert sum(fr["dp_table_exchange_steps"].values()) == 4
    if config == "c4":
        assert rec["config"]["embed_dim"] == 128 and rec["config"]["layer_size"] == [128, 64, 32]


def test_bench_c5_eight_ranks_gloo_rehearsal():
    """bench.py --gpus 8 --config c5 end to end at a tiny scale, all eight ranks on this one GPU
    over gloo -- shard_bounds with 8 cuts, the N mod 8 tail rows, the 7-peer all-peer gathers of the pipelined
    forward and the hop backward, the global-batch BPR -- with the frontier leg bit-identical to the
    whole-shard step on every rank (the row-sharded path the driver's 8-GPU run takes, minus RCCL)."""
    import json
    import subprocess
    import sys

    env = dict(os.environ, KGAT_BENCH_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = _run_logged([sys.executable, str(ROOT / "bench.py"), "--gpus", "8", "--config", "c5", "--scale", "0.0005",
                     "--steps", "2", "--warmup", "1"], env, "bench_c5_world8_gloo", timeout=400)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 8 and rec["config"]["parallelism"] == "row-sharded x8"
    rows = rec["config"]["shard_rows"]
    assert len(rows) == 8 and sum(rows) == rec["config"]["nodes"] and min(rows) > 0
    assert rec["rehearsal"].startswith("gloo") and rec["value"] > 0 and np.isfinite(rec["final_loss"])
    assert rec["frontier_forward"]["bit_identical_to_full"]["pass"] is True, rec["frontier_forward"]


def test_bench_c5_rank_share_small():
    """bench.py --rank-share K (one process, rank 0 of K alone: its rows of A / A^T, the full gathered layer
    buffers, the global batch from simulated peers, every collective local) at a tiny C5 scale: one JSON line
    with the share's shapes and HBM high-water mark, and a finite loss."""
    import json
    import subprocess
    import sys

    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--config", "c5", "--scale", "0.002", "--rank-share", "4",
                        "--steps", "2", "--warmup", "1", "--no-cpu-baseline"], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout
    rec = json.loads(lines[0])
    rs = rec["rank_share"]
    assert rec["n_gpus"] == 1 and rs["ranks"] == 4 and rs["rank"] == 0
    assert 0 < rs["shard_rows"] < rec["config"]["nodes"] and rs["shard_nnz_A"] > 0
    assert 0 < rs["hbm_peak_bytes"] and rec["value"] > 0 and np.isfinite(rec["final_loss"])
    assert rec["frontier_forward"]["bit_identical_to_full"]["pass"] is None  # not checkable in a share
