"""Multi-process (gloo, CPU) tests of the device data plane: collectives and the sharded
population sweep (rank 0 owns the experiment; C1 all-gather + C5 broadcast every sync)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch
    torch.set_num_threads(2)   # ranks share the host's CPUs (and pytest-xdist workers)
    from metaopt_amd.parallel.comm import init_from_env
    return init_from_env(backend="gloo")


def _collectives_worker(rank, world, port, q):
    comm = _init(rank, world, port)
    rows = torch.full((3, 2), float(rank))
    g = comm.all_gather_rows(rows)
    t = torch.tensor([7.0 if rank == 0 else 0.0])
    comm.broadcast_(t)
    s = torch.tensor([float(rank + 1)])
    comm.all_reduce_(s)
    mx = comm.max_float(rank * 2.5)
    if rank == 0:
        comm.send_tensor(torch.arange(4.0), dst=1)
        got = None
    else:
        got = comm.recv_tensor(torch.empty(4), src=0).tolist()
    q.put((rank, g[:, 0].tolist(), float(t), float(s), mx, got))
    dist.destroy_process_group()


def test_collectives_gloo():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_collectives_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for rank, gathered, b, s, mx, got in res:
        assert gathered == [0, 0, 0, 1, 1, 1]
        assert b == 7.0 and s == 3.0 and mx == 2.5
    assert res[1][5] == [0.0, 1.0, 2.0, 3.0]


def _sweep_worker(rank, world, port, q):
    comm = _init(rank, world, port)
    from metaopt_amd.io.experiment_builder import build_experiment
    from metaopt_amd.models.data import TeacherClassification
    from metaopt_amd.models.mlp import MLPSweepTask
    from metaopt_amd.ops.population import PopulationMLP
    from metaopt_amd.storage.database import EphemeralDB
    from metaopt_amd.storage.protocol import DocumentStorage
    from metaopt_amd.worker.population_sweep import PopulationSweep
    priors = {"/lr": "loguniform(1e-3, 1.0)", "/width": "loguniform(64, 128, discrete=True)",
              "/steps": "fidelity(16, 64, 2)"}
    exp = None
    if rank == 0:
        exp = build_experiment("dist-sweep", priors=priors,
                               algorithms={"asha": {"seed": 3, "repetitions": float("inf")}},
                               max_trials=20, storage=DocumentStorage(EphemeralDB()))
    data = TeacherClassification(n_train=512, n_val=128, batch_size=128, seed=1)
    pop = PopulationMLP(3, max_width=128, eval_batch=128, device="cpu")
    sweep = PopulationSweep(pop, MLPSweepTask(priors=priors, max_width=128), data, comm=comm,
                            experiment=exp, sync_every=16)
    summary = sweep.run(2000)
    sweep.close()
    statuses = None
    if rank == 0:
        statuses = [t.status for t in exp.fetch_trials()]
    q.put((rank, sweep.samples, summary["completed"], statuses, sweep.done))
    dist.destroy_process_group()


def test_sharded_sweep_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_sweep_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    (r0, samples0, done0, statuses, fin0), (r1, samples1, _, _, fin1) = res
    assert samples0 > 0 and samples1 > 0          # both ranks trained trials
    assert done0 == 20 and statuses.count("completed") == 20
    assert fin0 and fin1                          # both ranks saw the "done" flag


def _pbt_worker(rank, world, port, q):
    comm = _init(rank, world, port)
    import numpy as np
    from metaopt_amd.io.experiment_builder import build_experiment
    from metaopt_amd.models.data import TeacherClassification
    from metaopt_amd.models.mlp import MLPSweepTask
    from metaopt_amd.ops.population import PopulationMLP
    from metaopt_amd.storage.database import EphemeralDB
    from metaopt_amd.storage.protocol import DocumentStorage
    from metaopt_amd.worker.population_sweep import NEW, RESUME, AS_COLS, PopulationSweep
    priors = {"/lr": "loguniform(1e-3, 1.0)", "/width": "choices([64])",
              "/steps": "fidelity(16, 48, 2)"}
    exp = None
    if rank == 0:
        exp = build_experiment("dist-pbt", priors=priors,
                               algorithms={"pbt": {"seed": 3, "population_size": 6,
                                                   "interval": 16, "min_forking_population": 6,
                                                   "freeze": ["/width"]}},
                               storage=DocumentStorage(EphemeralDB()))
    data = TeacherClassification(n_train=512, n_val=128, batch_size=128, seed=1)
    pop = PopulationMLP(3, max_width=64, eval_batch=128, device="cpu")
    sweep = PopulationSweep(pop, MLPSweepTask(priors=priors, max_width=64), data, comm=comm,
                            experiment=exp, sync_every=16)
    # C4 directly: rank 0 holds a checkpoint that rank 1 resumes in its slot 2
    sweep.start()
    st = pop.slot_state(0)
    sweep.ckpts[999] = pop.save_states([(0, sweep._free_ck.pop())])[0]
    assign = np.zeros((2 * 3 + 1, AS_COLS))
    assign[3 + 2] = (RESUME, 0, 64, 0.1, 0.9, 0, 0, 7, 16, 999, 0, 0)
    got, direct = sweep._exchange_checkpoints(assign)
    assert not direct                         # the MLP population packs its state
    c4 = None
    if rank == 1:
        c4 = (sorted(got), got[2]["t"], got[2]["p32"].shape[0])
    ref = (int(st["t"]), st["p32"].shape[0], float(st["p32"].sum())) if rank == 0 else None
    sweep._free_ck.append(sweep.ckpts.pop(999)["ck"])
    summary = sweep.run(400)
    sweep.close()
    parents = None
    if rank == 0:
        trials = exp.fetch_trials()
        parents = (len(trials), sum(1 for t in trials if t.parents),
                   sum(1 for t in trials if t.status == "completed"))
    q.put((rank, c4, ref, parents, summary["completed"], sweep.done))
    dist.destroy_process_group()


def test_pbt_sweep_and_c4_copy_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_pbt_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    (r0, _, ref, parents, done0, fin0), (r1, c4, _, _, _, fin1) = res
    assert c4[0] == [2] and c4[1] == ref[0] and c4[2] == ref[1]
    n_trials, n_children, n_completed = parents
    assert n_trials == 18 and n_children == 12      # 6 members x 3 generations
    assert n_completed == 18 and fin0 and fin1


def _c4_flat_worker(rank, world, port, q, two=False):
    """C4 of a flat (CNN / LM) population: pool entry -> pool entry, no pack / unpack.  With
    ``two``, rank 1 receives two members in one sync with one reserved entry (P = 3 -> ceil(3/4)):
    the first lands in the pool, the second travels packed."""
    comm = _init(rank, world, port)
    import numpy as np
    from metaopt_amd.io.experiment_builder import build_experiment
    from metaopt_amd.models.resnet import PopulationResNet
    from metaopt_amd.ops.population import MemberConfig
    from metaopt_amd.storage.database import EphemeralDB
    from metaopt_amd.storage.protocol import DocumentStorage
    from metaopt_amd.worker.population_sweep import AS_COLS, RESUME, PopulationSweep
    from metaopt_amd.worker.tasks import get
    task = get("resnet20")
    exp = None
    if rank == 0:
        exp = build_experiment("dist-c4-flat", priors=dict(task.priors),
                               algorithms={"random": {"seed": 1}},
                               storage=DocumentStorage(EphemeralDB()))
    pop = PopulationResNet(3, batch_size=16, device="cpu", blocks_per_stage=1, image_size=16)
    pop.set_member(0, MemberConfig(width=0, lr=0.05, momentum=0.9, seed=11 + rank))
    pop.hp[0]["t"] = 5
    sweep = PopulationSweep(pop, task, data=None, comm=comm, experiment=exp, sync_every=8,
                            ckpt_capacity=4, pipelined=False)
    # both pools full: rank 0 sends its OLDEST checkpoint; the receive must not
    # evict anything on rank 1 (rank 0 mirrors every rank's FIFO without hearing of receives)
    keys = [999, 1000, 1001, 1002] if rank == 0 else [2000, 2001, 2002, 2003]
    for k in keys:
        sweep.ckpts[k] = pop.save_states([(0, sweep._free_ck.pop())])[0]
    assert not sweep._free_ck
    c4_free0 = len(sweep._c4_free)
    assign = np.zeros((2 * 3 + 1, AS_COLS))
    assign[3 + 2] = (RESUME, 0, 0, 0.1, 0.9, 0, 0, 7, 16, 999, 0, 0)
    if two:
        assign[3 + 1] = (RESUME, 0, 0, 0.1, 0.9, 0, 0, 7, 16, 1000, 0, 0)
    assert sweep._c4_reserve == 1 and len(sweep._c4_free) == 1
    states, metas = sweep._exchange_checkpoints(assign)
    out = None
    assert list(sweep.ckpts) == keys                    # nothing evicted on either rank
    if two:
        if rank == 1:
            assert sorted(metas) == [1] and sorted(states) == [2]
            pop.load_states([(1, metas[1])])
            pop.load_slot_state(2, states[2])
            out = (float(pop.slot_state(1)["p32"].double().sum()),
                   float(pop.slot_state(2)["p32"].double().sum()))
        else:
            s = float(pop.slot_state(0)["p32"].double().sum())
            out = (s, s)
        q.put((rank, out))
        dist.destroy_process_group()
        return
    if rank == 1:
        assert not states and sorted(metas) == [2]
        assert metas[2]["ck"] not in [m["ck"] for m in sweep.ckpts.values()]
        pop.load_states([(2, metas[2])])
        out = (metas[2]["t"], float(pop.slot_state(2)["p32"].double().sum()),
               len(sweep._c4_free) == c4_free0 - 1)
    else:
        out = (5, float(pop.slot_state(0)["p32"].double().sum()), True)
    q.put((rank, out))
    dist.destroy_process_group()


def test_c4_flat_population_pool_to_pool_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_c4_flat_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res[1][0] == res[0][0] == 5                  # step count travelled in the header
    assert res[1][1] == res[0][1]                       # the member's weights, bit for bit
    assert res[1][2]                                    # received into a pool entry


def test_c4_receives_past_the_reserve_travel_packed_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_c4_flat_worker, args=(r, world, port, q, True))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res[1] == res[0]        # both members arrive bit for bit (direct and packed)


# ------------------------------------------------------------------ launcher (no HIP before spawn)
def _fake_kfd(root, simds):
    for i, s in enumerate(simds):
        d = root / str(i)
        d.mkdir(parents=True)
        (d / "properties").write_text(f"cpu_cores_count {0 if s else 8}\nsimd_count {s}\n"
                                      f"gfx_target_version {90500 if s else 0}\n")
    return str(root)


def test_visible_gpu_count_from_kfd_topology(tmp_path):
    from metaopt_amd.parallel.launch import visible_gpu_count
    root = _fake_kfd(tmp_path / "nodes", [0, 1024, 1024, 1024, 1024])   # one CPU, four GPUs
    assert visible_gpu_count({}, root) == 4
    assert visible_gpu_count({"HIP_VISIBLE_DEVICES": "0,2"}, root) == 2
    assert visible_gpu_count({"ROCR_VISIBLE_DEVICES": "1", "HIP_VISIBLE_DEVICES": "0,1"}, root) == 1
    assert visible_gpu_count({"CUDA_VISIBLE_DEVICES": "-1"}, root) == 0
    assert visible_gpu_count({}, str(tmp_path / "absent")) == 0
    assert visible_gpu_count({"MOPT_GPU_COUNT": "2"}, str(tmp_path / "absent")) == 2


def test_visible_gpu_count_skips_inaccessible_render_nodes(tmp_path):
    """a container given some of the host's render nodes still sees every GPU in
    sysfs; only GPUs whose /dev/dri/renderD<minor> this process can open are counted."""
    from metaopt_amd.parallel.launch import visible_gpu_count
    root = _fake_kfd(tmp_path / "nodes", [0, 1024, 1024, 1024])
    for i, minor in ((1, 128), (2, 136), (3, 144)):
        with open(tmp_path / "nodes" / str(i) / "properties", "a") as f:
            f.write(f"drm_render_minor {minor}\n")
    dri = tmp_path / "dri"
    dri.mkdir()
    (dri / "renderD128").write_text("")
    (dri / "renderD144").write_text("")
    assert visible_gpu_count({}, root, str(dri)) == 2


def test_launcher_never_imports_torch_before_spawning():
    """rank_env (what bench.py / ``mopt sweep --gpus N`` run before starting the ranks) must not
    initialise HIP: it may not even import torch."""
    import subprocess
    import sys
    code = ("import sys; from metaopt_amd.parallel.launch import rank_env; env = rank_env(2); "
            "print(int('torch' in sys.modules), env['WORLD_SIZE'])")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                         timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.split() == ["0", "2"]
