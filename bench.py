#!/usr/bin/env python3
"""Benchmark: env-steps/s at 65 536 concurrent 4-player games per MI355X.

Driver contract: `python bench.py --gpus N --steps K --warmup W` (N>1 under
torch.distributed.run, one rank per GPU).  Prints ONE JSON line on rank 0.

Workload (BASELINE.json configs[1]): per GPU,
B = 65 536 independent 4-player games of DrunkHamster self-play in
numpy-compat RNG mode (game g replays np.random.seed(g) +
GameSession(DrunkHamster() x 4) of the reference, episode after episode).
One bench step = one rollout call that advances every game by one full
episode (10 env-steps: policy draw, simultaneous-play resolution, scoring,
per-seat int8 observation, auto-reset deal) and writes the whole trajectory
(obs, actions, rewards, done) to HBM: in numpy mode k_play (the game loop,
drawing from an LDS copy of pre-twisted MT19937 words) with, on a side
stream and concurrently, k_mt_ahead twisting every game's stream ~600 words
ahead for the next launch.  Inputs are resident on the device before timing
starts; the timed region includes both kernels.

Multi-GPU: game shards are independent (rank r owns global games
[r*B, (r+1)*B), streams keyed by the global id), so there is no collective
on the data path; one RCCL all_reduce of the per-rank score sums after the
timed loop is the score gather.

Extra legs (reported beside the headline, never in `value`): config 3
(MCS), config 4 (PUCT, PUCTCustomed), and config 5 on every rank: the
batched tournament (league.py) -- 65 536 concurrent tournament slots per GPU
with per-game seat draws, then the RCCL gather of the per-agent sums and
every game's record and the rank-0 Elo replay.
"""
import argparse
import json
import os
import sys
import subprocess
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "rl-6-nimmt_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
N_PLAYERS = 4
STEPS_PER_LAUNCH = 10
# algorithmic bytes per env-step at N players = 33N + 57
# (state round trip: hands 10N, board 24, lens 4, scores 4N, actions N read;
# hands, board, lens, scores, rewards 4N, done 1 written) + 47N for the int8
# observation the step emits.
ALGO_BYTES_PER_STEP = (33 * N_PLAYERS + 57) + 47 * N_PLAYERS  # 377 B at N = 4
# HBM bytes per bench step from rocprofv3 PMC passes of its kernels (numpy
# mode: k_mt_ahead + k_play; philox: k_play) -- tools/pmc_config2.sh: FETCH_SIZE
# and WRITE_SIZE in separate passes, gfx950 corrections of MI355X_MICROARCH.md
# applied by tools/pmc_traffic.py.  PMC counters cannot be read inside a plain
# run, so the committed summary of the current kernels is reported beside the
# live timing.
LIB_TWIST_EVERY = 4  # the library's SN_OPT_TWIST_EVERY default (include/sechs.h)
SQ_CONFIG4_ROLLOUTS = "profiles/r06_sq_config4_rollouts.json"  # SQ pass of k_puct_rollouts (eager launches)
PMC_TRAFFIC = {"numpy": os.path.join(ROOT, "profiles", "r06_final3_pmc_traffic_numpy.json"),  # tools/r06_final.sh
               "numpy_ring": os.path.join(ROOT, "profiles", "r06_base_pmc_traffic_numpy.json"),  # --pipe-dec 0
               "philox": os.path.join(ROOT, "profiles", "r04_pmc_traffic_philox.json")}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs of this node, one rank each (default: WORLD_SIZE, else 1); without a launcher, N > 1 "
                         "starts torch.distributed.run over N ranks as a child process")
    ap.add_argument("--steps", type=int, default=200, help="timed launches (episodes)")
    ap.add_argument("--warmup", type=int, default=20,
                    help="untimed launches first (several twist groups: the pipeline in its steady state)")
    ap.add_argument("--games", type=int, default=65536, help="games per GPU")
    ap.add_argument("--rng", default="numpy", choices=["numpy", "philox"])
    ap.add_argument("--no-obs", action="store_true", help="do not emit observations (not the headline)")
    ap.add_argument("--pipe-gpw", type=int, default=64, choices=[32, 64], help="games per k_play wave (pipelined path)")
    ap.add_argument("--play-split", type=int, default=None, choices=[0, 1],
                    help="SN_OPT_PLAY_SPLIT (default: the library's)")
    ap.add_argument("--twist-round", type=int, default=None, choices=[0, 1],
                    help="SN_OPT_TWIST_ROUND: whole-round MT19937 twists in k_mt_ahead (default: the library's, 1)")
    ap.add_argument("--launches-per-call", type=int, default=4,
                    help="bench steps (launches of 10 env-steps) per sn_rollout call in the timed loop: each writes "
                         "its own slice of a [10 x n]-step output (A/B of the host's per-call cost)")
    ap.add_argument("--pipe-dec", type=int, default=None, choices=[0, 1],
                    help="SN_OPT_PIPE_DEC: decode-ahead records (k_decode) for k_play (default: the library's, 1)")
    ap.add_argument("--twist-every", type=int, default=None, choices=[1, 2, 3, 4, 5],
                    help="SN_OPT_TWIST_EVERY: one k_mt_ahead per 1 .. 5 play launches (default: the library's)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-philox", action="store_true", help="skip the philox-mode leg of config 2")
    ap.add_argument("--no-mcs", action="store_true", help="skip the config-3 MCS leg")
    ap.add_argument("--mcs-games", type=int, default=8192)
    ap.add_argument("--mcs-rollouts", type=int, default=256)
    ap.add_argument("--no-puct", action="store_true", help="skip the config-4 PUCT leg")
    ap.add_argument("--no-league", action="store_true", help="skip the config-5 batched tournament leg")
    ap.add_argument("--no-scalar", action="store_true", help="skip the config-1 scalar drop-in leg")
    ap.add_argument("--league-rounds", type=int, default=10, help="timed tournament games per slot (config 5)")
    ap.add_argument("--no-mixed-league", action="store_true", help="skip the run.py-seated config-5 league leg")
    ap.add_argument("--mixed-slots", type=int, default=65536, help="tournament slots per GPU of the run.py league")
    ap.add_argument("--mixed-mc-max", type=int, default=200, help="mc_max of the run.py league's search agents")
    ap.add_argument("--no-dropin", action="store_true", help="skip the drop-in GameSession / Tournament search legs")
    ap.add_argument("--only", default="", help="comma list of legs to run (headline,cpu,mcs,puct,scalar,league,"
                                             "mixed,dropin,philox); empty = all")
    ap.add_argument("--puct-games", type=int, default=8192)
    return ap.parse_args()


def launch_ranks(n):
    """`python bench.py --gpus N` without a launcher (N > 1): run this same
    command under torch.distributed.run, one rank per GPU on this node, as a
    child process -- started before this process touches the GPU (no exec
    from a process that has) -- and hand back its exit code; rank 0 of the
    child prints the JSON line to the inherited stdout."""
    import socket

    try:
        avail = torch.cuda.device_count()  # does not initialise the GPU on this image
    except Exception:
        avail = None
    if avail is not None and avail < n and not os.environ.get("SECHS_BENCH_SHARED_GPU"):
        # SECHS_BENCH_SHARED_GPU=1: rehearse the N-rank path on fewer GPUs
        # (ranks share the visible devices; RCCL itself refuses two ranks on
        # one GPU, SECHS_BENCH_BACKEND=gloo runs the whole path)
        raise SystemExit(f"bench: --gpus {n} but {avail} GPU(s) visible (one rank per GPU)")
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def resolve_world(args):
    """(ranks to use, True when this process must launch them itself)"""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if args.gpus is not None and args.gpus != int(env_world):
            raise SystemExit(f"bench: --gpus {args.gpus} but the launcher started WORLD_SIZE={env_world} ranks")
        return int(env_world), False
    n = 1 if args.gpus is None else int(args.gpus)
    if n < 1:
        raise SystemExit("bench: --gpus must be >= 1")
    return n, n > 1


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        # SECHS_BENCH_BACKEND=gloo: rehearsal of the N-rank path with several
        # ranks sharing the visible GPUs (RCCL needs one GPU per rank); the
        # driver's runs use the default, nccl (= RCCL), one GPU per rank
        backend = os.environ.get("SECHS_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dev = local % torch.cuda.device_count() if os.environ.get("SECHS_BENCH_SHARED_GPU") else local
            torch.cuda.set_device(dev)
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            torch.cuda.set_device(local % torch.cuda.device_count())
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    return world, rank, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist

        dist.barrier()


ENQUEUE_S = None


def time_rollouts(env, out, steps, warmup, world, per_call=1):
    """Warm up, then time exactly `steps` launches between barrier+sync on
    both sides (nothing else enqueued in between: per-launch timing events
    on the stream cost the pipelined step ~30 %).  Returns (wall seconds,
    mean per-launch ms from HIP events around each launch in a second pass of
    the same `steps` launches, per-kernel times)."""
    one = {k: v[:STEPS_PER_LAUNCH] for k, v in out.items()}  # one launch's outputs
    for _ in range(warmup):
        env.rollout(STEPS_PER_LAUNCH, out=one)
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if per_call == 1:
        for i in range(steps):
            env.rollout(STEPS_PER_LAUNCH, out=one)
    else:  # n launches per call, each into its own slice of the [10 n]-step output
        for i in range(0, steps, per_call):
            n = min(per_call, steps - i) * STEPS_PER_LAUNCH
            env.rollout(n, out={k: v[:n] for k, v in out.items()})
    global ENQUEUE_S
    ENQUEUE_S = time.perf_counter() - t0  # host time to enqueue the timed launches (host-bound if ~ the wall)
    torch.cuda.synchronize()
    barrier(world)
    t1 = time.perf_counter()
    # second pass: HIP events around each launch on the launch stream, and
    # (numpy mode) inside the library around each kernel on its own stream --
    # over at least KERNEL_PASS_MIN launches (a 20-launch pass is dominated by
    # its first groups: k_play 70-75 vs 57-59 us steady, gpurun_out/r06_drv1)
    n2 = max(steps, KERNEL_PASS_MIN)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n2)]
    if env.rng == "numpy":
        env.time_kernels(n2)
    for i in range(n2):
        ev[i][0].record()
        env.rollout(STEPS_PER_LAUNCH, out=one)
        ev[i][1].record()
    torch.cuda.synchronize()
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    if env.rng != "numpy":
        return t1 - t0, kern_ms, {"k_play": kern_ms, "launches": n2}
    play_ms, ahead_ms, dec_ms, n = env.kernel_times(with_decode=True)
    env.time_kernels(0)
    return t1 - t0, kern_ms, {"k_play": play_ms, "k_mt_ahead": ahead_ms, "k_decode": dec_ms, "launches": n}


def make_out(env, games, with_obs, launches=1):
    T, B, N = STEPS_PER_LAUNCH * launches, games, N_PLAYERS
    dev = env.device
    out = {
        "rewards": torch.empty((T, B, N), dtype=torch.int32, device=dev),
        "done": torch.empty((T, B), dtype=torch.uint8, device=dev),
        "actions": torch.empty((T, B, N), dtype=torch.uint8, device=dev),
    }
    if with_obs:
        out["obs"] = torch.empty((T, B, N, 48), dtype=torch.int8, device=dev)
    return out


def cpu_baseline(budget_s, rng):
    """The oracle's C restatement of env.py + DrunkHamster (oracle/, kind
    "port"), single thread, on a bounded sample of the same workload."""
    from oracle import oracle as O

    mode = O.RNG_NUMPY_MT if rng == "numpy" else O.RNG_PHILOX
    # calibrate on a small batch, then size the sample to ~budget_s seconds
    B = 2048
    v = O.VecOracle(B, N_PLAYERS, rng_mode=mode, seed=0)
    v.reset()
    t = time.perf_counter()
    v.rollout(STEPS_PER_LAUNCH, want_obs=True, want_actions=True, nthreads=1)
    dt = time.perf_counter() - t
    per_game_ep = dt / B
    games = int(max(256, min(65536, budget_s / max(per_game_ep, 1e-9) / 2)))
    episodes = max(1, int(budget_s / (per_game_ep * games)))
    v = O.VecOracle(games, N_PLAYERS, rng_mode=mode, seed=0)
    v.reset()
    t = time.perf_counter()
    for _ in range(episodes):
        v.rollout(STEPS_PER_LAUNCH, want_obs=True, want_actions=True, nthreads=1)
    dt = time.perf_counter() - t
    steps = games * episodes * STEPS_PER_LAUNCH
    # the same restatement with OpenMP over this job's CPU share (SURVEY.md
    # §8(d)), ~3 s on the full 65 536 games: as many threads as this process
    # may run on, capped by OMP_NUM_THREADS when the job sets it
    host = host_cpu_info()
    threads = host["affinity_cpus"]
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        threads = max(1, min(threads, int(os.environ["OMP_NUM_THREADS"])))
    vm = O.VecOracle(65536, N_PLAYERS, rng_mode=mode, seed=0)
    vm.reset()
    vm.rollout(STEPS_PER_LAUNCH, want_obs=True, want_actions=True, nthreads=threads)  # first touch of the outputs
    t = time.perf_counter()
    eps_mt = 0
    while eps_mt == 0 or time.perf_counter() - t < 3.0:
        vm.rollout(STEPS_PER_LAUNCH, want_obs=True, want_actions=True, nthreads=threads)
        eps_mt += 1
    dt_mt = time.perf_counter() - t
    return {
        "value": steps / dt,
        "unit": "env-steps/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{games} games x {episodes} episodes x 10 env-steps ({steps} env-steps, {dt:.1f} s) of the same "
                  f"workload (DrunkHamster self-play, {rng} RNG, int8 obs + actions + rewards written) on the "
                  f"oracle's single-threaded C restatement of env.py",
        "multi_thread": {"value": 65536 * eps_mt * STEPS_PER_LAUNCH / dt_mt, "cores": threads,
                         "sample": f"65536 games x {eps_mt} episodes, OpenMP"},
        "host": host,
    }


def host_cpu_info():
    """What the CPU baseline ran on: logical CPUs of the machine, the CPUs
    this process may use (its affinity mask, the job's share on the GPU box),
    OMP_NUM_THREADS, and the CPU model (lscpu / /proc/cpuinfo)."""
    model = None
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                model = line.split(":", 1)[1].strip()
                break
    except (OSError, subprocess.SubprocessError):
        pass
    if model is None:
        try:
            for line in open("/proc/cpuinfo"):
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
        except OSError:
            pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    return {"cpu_model": model, "os_cpu_count": os.cpu_count(), "affinity_cpus": aff,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


# VALU issue peak of MI355X: 256 CUs x 4 SIMD-32, one wave64 VALU
# instruction per 2 cycles each (MI355X_MICROARCH.md "Wave scheduling"), at
# the 2.4 GHz peak engine clock
VALU_PEAK_GINSTR = 256 * 4 * 2.4 / 2  # 1228.8 G wave-instructions/s
CLOCK_HZ = 2.4e9  # the peak engine clock
KERNEL_PASS_MIN = 100  # launches in the per-kernel timing pass (outside the timed region)
SQ_EXTRAS = os.path.join(ROOT, "profiles", "r04_sq_extras.json")


def sq_extras(kernel):
    """SQ counters of the config-3/4 kernels, summed over one run of the legs
    (tools/r04_prof2.sh -> profiles/r04_sq_extras.json; config 3 only: the PMC pass over the
    graph-replayed config-4 leg crashes rocprofv3 on this image)"""
    if not os.path.exists(SQ_EXTRAS):
        return None
    for name, c in json.load(open(SQ_EXTRAS)).items():
        if kernel in name:
            return c
    return None


def bench_mcs(games, rollouts, episodes=1):
    """BASELINE config 3: every seat of `games` 4-player games is an MCS
    agent with `rollouts` playouts per legal move (stratified), one whole
    game (10 decisions per seat, 9 of them searched) per episode.  Unit:
    playout env-steps (one playout game advancing one turn)."""
    from rl_6_nimmt.mcs import BatchedMCS, rollout_env_steps_per_seat_game
    from rl_6_nimmt.vec_env import VecSechsNimmtEnv

    env = VecSechsNimmtEnv(games, N_PLAYERS, seed=1, rng="philox")
    mcs = BatchedMCS(env, rollouts=rollouts, seed=2)
    mcs.play_episode()  # warm-up
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    total = None
    for _ in range(episodes):
        total = mcs.play_episode()
    ev1.record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    steps = rollout_env_steps_per_seat_game(rollouts) * N_PLAYERS * games * episodes
    decisions = 9 * N_PLAYERS * games * episodes
    gpu_ms = ev0.elapsed_time(ev1)
    sq = sq_extras("k_mcs_rollouts")
    roof = None
    if sq and episodes == 1 and games == 8192 and rollouts == 256:
        # the search is integer VALU work (no HBM traffic to speak of: 189 B
        # per playout env-step by the SURVEY model, ~0 real); bound = VALU issue
        # the profiled run (tools/extras_only.py) is bench_mcs itself: the
        # warm-up episode + the timed one, so half the counted instructions
        valu = sq["SQ_INSTS_VALU"] / 2
        achieved = valu / (gpu_ms * 1e-3) / 1e9
        roof = {"bound": "valu", "achieved": achieved, "peak": VALU_PEAK_GINSTR, "unit": "G wave-instr/s",
                "frac": achieved / VALU_PEAK_GINSTR, "traffic": None,
                "valu_instructions": valu, "valu_source": os.path.relpath(SQ_EXTRAS, ROOT),
                "wave_cycles": {k: sq.get(k + "_frac") for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY")},
                "kernel": "k_mcs_rollouts<4> (+ memorize/choose), over the episode's GPU time (HIP events)"}
    return {
        "workload": f"config3: {games} x 4-player games, all seats MCS, {rollouts} playouts per legal move, "
                    f"{episodes} game(s); philox RNG",
        "value": steps / wall,
        "unit": "playout env-steps/s",
        "decisions_per_s": decisions / wall,
        "wall_s": wall,
        "gpu_ms": gpu_ms,
        "roofline": roof,
        "mean_score_per_seat": (total.double().mean(dim=0)).tolist(),
    }


def bench_puct(games, mc_max=100, mc_per_card=10):
    """BASELINE config 4: Alpha0.5 (PUCT) self-play, every seat of `games`
    4-player games searches with the reference's defaults (mc_max=100,
    mc_per_card=10, c_puct=2); the policy MLP runs in bf16 through
    PyTorch-ROCm.  One whole game per measurement.  Units: playout env-steps
    (one rollout game advancing one turn) and policy rows (one candidate
    move scored, 2*(48*100+100*100+100) = 29 800 FLOP)."""
    from rl_6_nimmt.puct import BatchedPUCT, make_actor
    from rl_6_nimmt.vec_env import VecSechsNimmtEnv

    env = VecSechsNimmtEnv(games, N_PLAYERS, seed=3, rng="philox")
    torch.manual_seed(0)
    eng = BatchedPUCT(env, make_actor(), mc_per_card=mc_per_card, mc_max=mc_max, seed=4, net_dtype=torch.bfloat16,
                      graph=True)
    env.reset()
    eng.play_episode()  # warm-up: kernels, GEMM heuristics, one hipGraph capture per hand size
    env.reset()
    torch.cuda.synchronize()
    eng.rows_evaluated = 0
    t0 = time.perf_counter()
    total = eng.play_episode()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    steps = sum(eng.n_mc(n) * n for n in range(2, 11)) * N_PLAYERS * games
    rows_s = eng.rows_evaluated / wall
    fused = eng._net is not None and eng._net.fused() is not None
    whole = fused and eng.fused_rollouts and eng.deal_batch > 0  # sn_puct_rollouts
    tflops = eng.rows_evaluated * 29800 / wall / 1e12
    sq4 = None  # SQ counters of the rollout MLP kernel (eager launches)
    try:
        if whole:
            src = SQ_CONFIG4_ROLLOUTS
            c = json.load(open(os.path.join(ROOT, src)))["void k_puct_rollouts<4, 4>"]
        else:
            src = "profiles/r04_sq_config4_kernels.json"
            c = json.load(open(os.path.join(ROOT, src)))["k_puct_mlp_seats"]
        busy = c["SQ_VALU_MFMA_BUSY_CYCLES"] / c["dispatches_per_pass"]
        sq4 = {"mfma_busy_cycles_per_launch": busy,
               "valu_per_wave": c["SQ_INSTS_VALU_per_wave"], "mfma_per_wave": c["SQ_INSTS_MFMA"] / c["SQ_WAVES"],
               "valu_per_mfma": c["SQ_INSTS_VALU"] / c["SQ_INSTS_MFMA"], "source": src}
        if c.get("kernel_avg_ns"):
            # MFMA-busy SIMD-cycles over the launch's SIMD-cycles (256 CUs x 4 SIMDs) at the 2.4 GHz peak clock
            # (a lower clock would give a higher fraction)
            sq4["mfma_busy_frac"] = busy / (1024 * c["kernel_avg_ns"] * 1e-9 * CLOCK_HZ)
            sq4["kernel_avg_ns"] = c["kernel_avg_ns"]
    except (OSError, KeyError, ValueError, ZeroDivisionError):
        pass
    if fused:
        # the rollout MLP runs in one MFMA kernel: no activation tensor in
        # HBM; priced as the reference's 29 800 FLOP per candidate row
        # against the dense bf16 MFMA peak, over the whole game's wall time
        # (every kernel included)
        roof = {"bound": "mfma", "achieved": tflops, "peak": 2500.0, "unit": "TFLOP/s", "frac": tflops / 2500.0,
                "traffic": None, "algo_flop_per_row": 29800, "sq": sq4,
                "kernel": ("whole rollouts = sn_puct_deal_batch (16 rollouts' deals) + sn_puct_rollouts (one wave "
                           "per group of 8 decisions: every step's seat rows, MFMA layer 1 + 2 and head into logits "
                           "in LDS, the seat-lane step; two waves per SIMD); whole-game wall time") if whole
                else ("rollout step = sn_puct_mlp_seats (MFMA: seat rows, layer 1 per seat, card column, "
                      "layer 2, head in one persistent kernel) + k_puct_step_seats; whole-game wall time")}
    else:
        # any other net: candidate rows + the net's PyTorch-ROCm forward (hipBLASLt GEMMs),
        # HBM-bound on their bf16 intermediates -- per row 96 B in, 2 x (200 B out + 200 B
        # back in), 32 B head out = 928 B
        row_bytes = 96 + 2 * (200 + 200) + 32
        roof = {"bound": "hbm", "achieved": rows_s * row_bytes / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": rows_s * row_bytes / 1e9 / HBM_PEAK_GBS, "traffic": None, "algo_bytes_per_row": row_bytes,
                "mfma_frac": tflops / 2500.0,
                "kernel": "policy MLP (PyTorch-ROCm hipBLASLt bf16), whole game wall time incl. the k_puct_* kernels"}
    return {
        "workload": f"config4: {games} x 4-player games, all seats PUCT (mc_max={mc_max}, mc_per_card={mc_per_card}, "
                    f"c_puct=2), bf16 policy MLP 48-100-100-1 ("
                    + ("whole rollouts in one MFMA kernel" if whole else "one MFMA kernel per rollout step" if fused
                       else "PyTorch-ROCm GEMMs")
                    + f"), 1 game; each decision's rollout "
                    f"chain replayed from a captured hipGraph",
        "value": steps / wall,
        "unit": "playout env-steps/s",
        "decisions_per_s": 9 * N_PLAYERS * games / wall,
        "policy_rows_per_s": rows_s,
        "policy_tflops": tflops,
        "mlp": "whole rollouts (sn_puct_rollouts)" if whole else "fused, one kernel (sn_puct_mlp_seats)" if fused
        else "rows + PyTorch GEMMs",
        "roofline": roof,
        "wall_s": wall,
        "mean_score_per_seat": total.double().mean(dim=0).tolist(),
    }


def bench_league(world, rank, slots, rounds, warmup=2, K=5, lo=2, hi=4):
    """BASELINE config 5: tournament.py self-play sharded over the ranks.
    Rank r plays global slots [r*slots, (r+1)*slots); slot g is the
    reference's np.random.seed(g) + Tournament(2, 4) over 5 DrunkHamster
    agents + play_game() repeatedly (seat draw, deal, moves in-kernel; golden
    F11 pins it).  Timed: `rounds` games per slot (10 env-steps each) on every
    rank.  Then the RCCL score gather: all_reduce of the per-agent sums and
    all_gather of every game's record, Elo replayed on rank 0 (host C++) in
    canonical order -- timed separately."""
    from rl_6_nimmt.distributed import backend_label, gather_league_records, max_over_ranks, reduce_agent_stats
    from rl_6_nimmt.league import BatchedTournament, replay_league_elo

    t = BatchedTournament(slots, lo, hi, seed=0, game_offset=rank * slots, rng="numpy")
    for i in range(K):
        t.add_player(f"DrunkHamster_{i}")
    t.play_games(warmup)
    t.agent_stats()  # first use of the scoring kernels, outside the timing
    t.clear_records()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(rounds):
        t.play_games(1)
    torch.cuda.synchronize()
    barrier(world)
    wall = time.perf_counter() - t0
    if t.env.pipe_errors():
        raise SystemExit("bench: tournament draws ran past the twisted words")
    tg = time.perf_counter()
    # per-rank sums (host float64) and device records: the helpers place each
    # on the device the group's backend takes (RCCL: the GPU)
    from rl_6_nimmt.league import league_agent_stats

    timed = t.all_records()  # the timed rounds only
    stats = reduce_agent_stats(league_agent_stats(timed, K, hi))
    allrec = gather_league_records(timed, dst=0)  # the Elo replay runs on rank 0 only
    torch.cuda.synchronize()
    gather_ms = (time.perf_counter() - tg) * 1e3
    if world > 1:
        wall, gather_ms = max_over_ranks([wall, gather_ms], device=t.env.device)
    out = None
    if rank == 0:
        te = time.perf_counter()
        elos = replay_league_elo(allrec, K, hi)
        elo_ms = (time.perf_counter() - te) * 1e3
        s = stats.cpu().numpy()
        games = world * slots * rounds
        out = {
            "workload": f"config5: tournament.py self-play, {world} x {slots} concurrent game slots ({world * slots} "
                        f"games at once), {K} DrunkHamster agents, {lo}..{hi} players per game drawn per game, "
                        f"{rounds} games per slot; numpy-MT (slot g = np.random.seed(g) reference tournament)",
            "value": games * STEPS_PER_LAUNCH / wall,
            "unit": "env-steps/s",
            "games_per_s": games / wall,
            "concurrent_games": world * slots,
            "wall_s": wall,
            "ms_per_round": wall / rounds * 1e3,
            "score_gather_ms": gather_ms,
            "score_gather": f"{backend_label()} all_reduce of [{K}, 4] per-agent sums + gather to rank 0 of {games} "
                            f"game records ({allrec.numel() * 4 / 1e6:.1f} MB)" if world > 1 else "single rank (no collective)",
            "elo_replay_ms": elo_ms,
            "agents": {f"DrunkHamster_{i}": {"games": int(s[i, 0]), "mean_score": s[i, 1] / s[i, 0],
                                              "mean_position": s[i, 2] / s[i, 0], "win_fraction": s[i, 3] / s[i, 0],
                                              "elo": float(elos[i])} for i in range(K)},
        }
    t.close()
    return out


def run_py_league(mc_max=200, with_random=True):
    """the agents of run.py:24-27 (ACER minibatch 10, MCS / Alpha0.5 /
    Alpha0.5_customed at mc_max), all .train() as run.py:29-33 does, plus the
    DrunkHamster of the notebook's league (simple_tournament.ipynb)"""
    from rl_6_nimmt.agents import BatchedACERAgent, DrunkHamster, MCSAgent, PUCTAgent, PUCTCustomedAgent

    torch.manual_seed(0)
    agents = [("ACER", BatchedACERAgent(minibatch=10)), ("MCS", MCSAgent(mc_max=mc_max)),
              ("Alpha0.5", PUCTAgent(mc_max=mc_max)), ("Alpha0.5_customed", PUCTCustomedAgent(mc_max=mc_max))]
    if with_random:
        agents.append(("Random", DrunkHamster()))
    for _, a in agents:
        try:  # run.py:29-33: agents without parameters have no optimizer
            a.train()
        except ValueError:
            pass
    return agents


def bench_league_mixed(world, rank, slots, mc_max=200, rounds=1, warmup=1):
    """BASELINE config 5 with the reference's real league (run.py:20-40):
    ACER, MCS, Alpha0.5 (PUCT) and Alpha0.5_customed at mc_max=200 plus
    Random, Tournament(2, 4), training on, `slots` concurrent tournament games
    per GPU (slot g = np.random.seed(g) stream: seat draws, deals, Random and
    MCS seats in-kernel; the net agents' batched engines over their seats).
    Timed: `rounds` game rounds on every rank (each: every slot plays one
    whole game, then every net agent's batched update), then the RCCL
    gather of the per-agent sums and every game record + the rank-0 Elo
    replay."""
    from rl_6_nimmt.distributed import backend_label, gather_league_records, max_over_ranks, reduce_agent_stats
    from rl_6_nimmt.league import BatchedTournament, replay_league_elo

    # warm-up: `warmup` untimed rounds of the SAME league at full size, so
    # the timed round finds the handle, the engines, their buffers, the ACER
    # replay and every GEMM shape allocated and selected already (a fresh
    # league in the timed region measured 3.9-5.9 s per round, r03)
    specs = run_py_league(mc_max)
    t = BatchedTournament(slots, 2, 4, seed=0, game_offset=rank * slots, rng="numpy", train=True)
    for name, agent in specs:
        t.add_player(name, agent)
    for _ in range(warmup):
        t.play_games(1)
    t.agent_stats()
    for e in t.engines.values():
        e.rows_evaluated = 0
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    rec0 = len(t.records)
    t0 = time.perf_counter()
    for _ in range(rounds):
        t.play_games(1)
    torch.cuda.synchronize()
    barrier(world)
    wall = time.perf_counter() - t0
    rows = {n: e.rows_evaluated for n, e in t.engines.items()}  # the timed rounds only (reset after the warm-up)
    recs = torch.cat([r for r, _ in t.records[rec0:]], dim=0)
    # one more round with HIP events around its phases (outside the timed
    # region: where a round's time goes)
    t.phase_timing = True
    tp = time.perf_counter()
    t.play_games(1)
    torch.cuda.synchronize()
    phase_round_s = time.perf_counter() - tp
    phases = {"gpu_ms": {k: round(v, 2) for k, v in t.phase_ms.items()},
              "host_enqueue_ms": {k: round(v, 2) for k, v in t.phase_host_ms.items()},
              "round_wall_s": phase_round_s,
              "note": "a second, instrumented round: HIP events per phase on the stream (GPU ms) and the host's "
                      "enqueue time per phase; phases run back to back, so GPU ms sum to about the round"}
    tg = time.perf_counter()
    K = len(specs)
    from rl_6_nimmt.league import league_agent_stats

    stats = reduce_agent_stats(league_agent_stats(recs, K, 4))
    allrec = gather_league_records(recs, dst=0)  # the Elo replay runs on rank 0 only
    torch.cuda.synchronize()
    gather_ms = (time.perf_counter() - tg) * 1e3
    if world > 1:
        wall, gather_ms = max_over_ranks([wall, gather_ms], device=t.env.device)
    out = None
    if rank == 0:
        te = time.perf_counter()
        elos = replay_league_elo(allrec, K, 4)
        elo_ms = (time.perf_counter() - te) * 1e3
        s = stats.cpu().numpy()
        games = world * slots * rounds
        out = {
            "workload": f"config5 (run.py league): tournament.py self-play, {world} x {slots} concurrent game slots, "
                        f"agents ACER(minibatch=10), MCS, Alpha0.5 (PUCT), Alpha0.5_customed at mc_max={mc_max} + "
                        f"Random, 2..4 players drawn per game, training on (one batched Adam step per net agent per "
                        f"round); numpy-MT slot streams (slot g = np.random.seed(g)); {warmup} untimed round(s) of "
                        f"the same league, then {rounds} timed round(s)",
            "value": games * STEPS_PER_LAUNCH / wall,
            "unit": "env-steps/s",
            "games_per_s": games / wall,
            "s_per_round": wall / rounds,
            "concurrent_games": world * slots,
            "reference_s_per_game": [21.47, 46.95],
            "reference_source": "experiments/simple_tournament.ipynb:158-410 tqdm logs (CPU, one game at a time)",
            "policy_rows_per_round": {n: r / rounds for n, r in rows.items()},
            "phases": phases,
            "score_gather_ms": gather_ms,
            "score_gather": f"{backend_label()} all_reduce of [{K}, 4] per-agent sums + gather to rank 0 of {games} "
                            f"game records" if world > 1 else "single rank (no collective)",
            "elo_replay_ms": elo_ms,
            "agents": {n: {"games": int(s[i, 0]), "mean_score": s[i, 1] / max(1, s[i, 0]),
                           "win_fraction": s[i, 3] / max(1, s[i, 0]), "elo": float(elos[i])}
                       for i, (n, _) in enumerate(specs)},
        }
    t.close()
    return out


def bench_dropin(mcs_games=3, puct_games=3, tour_games=3, mc_max_tour=200):
    """The drop-in search path a reference user runs: s per
    game of GameSession(MCSAgent(), DrunkHamster() x 3) and GameSession(
    PUCTAgent() [training], DrunkHamster() x 3) -- SURVEY §6's cProfile setups,
    1.06-1.89 s and 11.6-14.7 s per game on this image's CPU -- and of a
    Tournament(2, 4) seated like run.py (the notebook's 21-47 s per game).
    One game at a time, the search on the GPU (reference-exact MCS lane,
    batched PUCT over one decision)."""
    from rl_6_nimmt import GameSession, Tournament
    from rl_6_nimmt.agents import DrunkHamster, MCSAgent, PUCTAgent

    def per_game(sess, n, warmup=1):
        for w in range(warmup):  # kernels; a PUCT agent's rollout graphs (captured at a shape's second use)
            np.random.seed(1000 + w)
            sess.play_game()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for g in range(n):
            np.random.seed(g + 1)
            sess.play_game()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n

    out = {}
    out["mcs_3random_s_per_game"] = per_game(GameSession(MCSAgent(), DrunkHamster(), DrunkHamster(), DrunkHamster()),
                                             mcs_games)
    out["mcs_reference_s_per_game"] = [1.06, 1.89]
    torch.manual_seed(0)
    puct = PUCTAgent()
    puct.train()
    out["puct_train_3random_s_per_game"] = per_game(GameSession(puct, DrunkHamster(), DrunkHamster(), DrunkHamster()),
                                                    puct_games, warmup=2)
    out["puct_reference_s_per_game"] = [11.6, 14.7]
    tour = Tournament(min_players=2, max_players=4)
    for name, agent in run_py_league(mc_max_tour, with_random=False):
        tour.add_player(name, agent)
    np.random.seed(0)
    tour.play_game()  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(tour_games):
        tour.play_game()
    torch.cuda.synchronize()
    out["run_py_tournament_s_per_game"] = (time.perf_counter() - t0) / tour_games
    out["tournament_reference_s_per_game"] = [21.47, 46.95]
    out["workload"] = (f"drop-in (one game at a time, host loop over the one-game device env): GameSession(MCSAgent() "
                       f"[mc_max 100], DrunkHamster x3) x {mcs_games}, GameSession(PUCTAgent() [mc_max 100, training], "
                       f"DrunkHamster x3) x {puct_games} after 2 untimed (its rollout graphs are captured at a shape's second "
                       f"decision), Tournament(2, 4) of run.py's agents at mc_max={mc_max_tour} "
                       f"(training) x {tour_games} games")
    out["reference_source"] = ("SURVEY.md §6 cProfile runs of the reference on this image's CPU (MCS, PUCT) and "
                               "experiments/simple_tournament.ipynb:158-410 (tournament)")
    return out


def bench_scalar(games=200, step_games=200):
    """BASELINE config 1 through the scalar drop-in (rl_6_nimmt.GameSession /
    SechsNimmtEnv on a one-game device handle, sn_step1 / sn_reset1): ms per
    GameSession(DrunkHamster(), DrunkHamster()) game (np.random.seed(g) per
    game, results bit-exact vs the reference's sessions, golden F2), and
    us per 4-player env.step with the actions drawn outside the timer -- the
    two reference numbers of BASELINE.md §2 (1.39 ms/game, 67.9 us/step on
    this image's CPU)."""
    from rl_6_nimmt import GameSession, SechsNimmtEnv
    from rl_6_nimmt.agents import DrunkHamster

    sess = GameSession(DrunkHamster(), DrunkHamster())
    np.random.seed(0)
    sess.play_game()  # warm-up (kernels, pinned buffers)
    t0 = time.perf_counter()
    for g in range(games):
        np.random.seed(g)
        sess.play_game()
    per_game = (time.perf_counter() - t0) / games
    env = SechsNimmtEnv(4, verbose=False)
    rng = np.random.RandomState(1)
    env.reset()
    step_s, steps = 0.0, 0
    for g in range(step_games):
        states, legal = env.reset()
        done = False
        while not done:
            acts = [int(rng.choice(h)) for h in legal]
            t = time.perf_counter()
            (states, legal), rew, done, _ = env.step(acts)
            step_s += time.perf_counter() - t
            steps += 1
    return {
        "workload": "config1: GameSession(DrunkHamster(), DrunkHamster()).play_game() through the scalar drop-in "
                    "(one-game device handle); 4-player env.step with actions drawn outside the timer",
        "ms_per_game": per_game * 1e3,
        "reference_ms_per_game": 1.39,
        "us_per_env_step_4p": step_s / steps * 1e6,
        "reference_us_per_env_step_4p": 67.9,
        "games": games,
        "steps_timed": steps,
    }


def bench_customed(games, episodes=5):
    """BASELINE config 4, policy/value-net variant: PUCTCustomedAgent
    (mcts.py:325-451) in every seat of `games` 4-player games -- per
    decision one 2-head MLP forward (bf16, PyTorch-ROCm) over the root
    candidates, the move = first argmax of the value head.  `episodes` whole
    games back to back; units: env-steps and decisions (one seat's move)."""
    from rl_6_nimmt.puct import BatchedPUCTCustomed, make_actor_value
    from rl_6_nimmt.vec_env import VecSechsNimmtEnv

    env = VecSechsNimmtEnv(games, N_PLAYERS, seed=3, rng="philox")
    torch.manual_seed(0)
    eng = BatchedPUCTCustomed(env, make_actor_value(), seed=4, net_dtype=torch.bfloat16)
    eng.play_episode()  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tot = None
    for _ in range(episodes):
        total, _ = eng.play_episode()
        tot = total if tot is None else tot + total
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    return {
        "workload": f"config4 (policy/value net): {games} x 4-player games, all seats PUCTCustomedAgent, bf16 2-head "
                    f"MLP 48-100-100-2 via PyTorch-ROCm, {episodes} games",
        "value": 10 * games * episodes / wall,
        "unit": "env-steps/s",
        "decisions_per_s": 10 * N_PLAYERS * games * episodes / wall,
        "wall_s": wall,
        "mean_score_per_seat": (tot.double() / episodes).mean(dim=0).tolist(),
    }


def bench_acer(games, episodes=3):
    """BatchedACERAgent (actor_critic.py:119-207) in every seat
    of `games` 4-player games -- per decision one 2-head MLP forward (bf16,
    PyTorch-ROCm) over the root candidates + the Philox sampler; after every
    game the reference's update schedule (one on-policy + one off-policy Adam
    step per flushed sequence; minibatch 2 sequences per decider) on the fp32
    rows of the device replay.  Times self-play and updates separately."""
    from rl_6_nimmt.acer import BatchedACER, make_actor_critic
    from rl_6_nimmt.vec_env import VecSechsNimmtEnv

    env = VecSechsNimmtEnv(games, N_PLAYERS, seed=3, rng="philox")
    torch.manual_seed(0)
    eng = BatchedACER(env, make_actor_critic().to(env.device), seed=4, net_dtype=torch.bfloat16, warmup=2,
                      minibatch=2, capacity=4)
    opt = torch.optim.Adam(eng.actor.parameters())
    for _ in range(3):  # fill the replay past warmup
        eng.play_episode()
        eng.learn(opt)
    play = learn = 0.0
    updates = 0
    for _ in range(episodes):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.play_episode()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        updates += len(eng.learn(opt))
        torch.cuda.synchronize()
        play, learn = play + t1 - t0, learn + time.perf_counter() - t1
    return {
        "workload": f"ACER: {games} x 4-player games, all seats BatchedACER (2-head MLP 48-100-100-(1,1) via "
                    f"PyTorch-ROCm: recording self-play samples from the fp32 training forward, Philox sampler), "
                    f"replay of 4 episodes, {episodes} timed games + updates",
        "value": 10 * games * episodes / play,
        "unit": "env-steps/s (self-play)",
        "decisions_per_s": 10 * N_PLAYERS * games * episodes / play,
        "updates": updates,
        "update_ms": 1e3 * learn / max(1, updates),
        "sequence_rows_per_s": (updates // 2) * 3 * N_PLAYERS * games * 10 / learn,
        "last_losses": list(eng.last_losses[-1]),
    }


def pmc_traffic(rng, games):
    """per-dispatch HBM bytes of the headline kernels from the committed
    rocprofv3 PMC passes (tools/pmc_traffic.py), and -- numpy mode -- the
    step traffic recomputed from the same file: each kernel's bytes per
    dispatch x its MEASURED dispatches per play launch in that run (the
    start-up twist k_mt_ahead<true, ..> excluded: once per pipeline start)"""
    path = PMC_TRAFFIC[rng]
    if games != 65536 or not os.path.exists(path):
        return None, None
    rec = json.load(open(path))
    per_kernel = {k: v["traffic_bytes_per_dispatch"] for k, v in rec["kernels"].items()}
    per_kernel["_ratio"] = {k: v.get("dispatches_per_play_launch") for k, v in rec["kernels"].items()}
    per_kernel["_step"] = sum(v["traffic_bytes_per_dispatch"] * v["dispatches_per_play_launch"]
                              for k, v in rec["kernels"].items()
                              if "dispatches_per_play_launch" in v and "k_mt_ahead<true" not in k) or None
    return per_kernel, os.path.relpath(path, ROOT)


def main():
    args = parse()
    n, spawn = resolve_world(args)
    if spawn:
        sys.exit(launch_ranks(n))
    world, rank, local = dist_setup(args)
    legs = set(x for x in args.only.split(",") if x)

    def want(leg):
        return not legs or leg in legs

    if legs and "headline" not in legs:  # profiling runs of single legs (tools/), not the driver's line
        result = {"legs": sorted(legs)}
        if want("mixed"):
            result["extra_config5_run_py_league"] = bench_league_mixed(world, rank, args.mixed_slots, args.mixed_mc_max)
        if want("dropin"):
            result["extra_dropin_search"] = bench_dropin()
        if want("puct"):
            result["extra_config4_puct"] = bench_puct(args.puct_games)
        if want("mcs"):
            result["extra_config3_mcs"] = bench_mcs(args.mcs_games, args.mcs_rollouts)
        if want("scalar"):
            result["extra_config1_scalar"] = bench_scalar()
        if want("acer"):
            result["extra_acer"] = bench_acer(args.puct_games // 2)
        if rank == 0:
            print(json.dumps(result), flush=True)
        return
    from rl_6_nimmt.vec_env import VecSechsNimmtEnv

    B = args.games
    env = VecSechsNimmtEnv(B, N_PLAYERS, seed=0, game_offset=rank * B, rng=args.rng)
    if args.rng == "numpy":
        env.set_option(pipe_gpw=args.pipe_gpw, play_split=args.play_split, twist_round=args.twist_round,
                       twist_every=args.twist_every, pipe_dec=args.pipe_dec)
    env.reset()
    out = make_out(env, B, not args.no_obs, args.launches_per_call)
    wall, kern_ms, kt = time_rollouts(env, out, args.steps, args.warmup, world, args.launches_per_call)

    # pipelined draws must never have run past the twisted words (checked
    # after the timed region; a nonzero count would void the parity claim)
    pipe_errors = env.pipe_errors() if args.rng == "numpy" else 0
    if pipe_errors:
        raise SystemExit(f"bench: {pipe_errors} pipelined MT19937 draws ran past the twisted words")
    # tournament score gather over RCCL (outside the timed region)
    sums, eps = env.results()
    tot = sums.to(torch.float64).sum(dim=0)
    if world > 1:
        from rl_6_nimmt.distributed import max_over_ranks, reduce_agent_stats

        wall, kern_ms, kt["k_play"], ahead = max_over_ranks([wall, kern_ms, kt["k_play"], kt.get("k_mt_ahead", 0.0)],
                                                           device=env.device)
        if "k_mt_ahead" in kt:
            kt["k_mt_ahead"] = ahead
        reduce_agent_stats(tot)

    total_steps = world * B * STEPS_PER_LAUNCH * args.steps
    value = total_steps / wall
    launch_steps = B * STEPS_PER_LAUNCH
    # dominant kernel = k_play (the game loop); its algorithmic bytes are the
    # SURVEY.md §8(d) 377 B per env-step x the 655 360 env-steps of a launch,
    # its duration the live HIP-event mean on its own stream (numpy mode: the
    # twist-ahead k_mt_ahead runs concurrently on a side stream and is
    # reported beside it; the whole step is `step_ms`)
    play_ms = kt["k_play"]
    twist_k = args.twist_every or LIB_TWIST_EVERY
    play_mode = ("RNG_PHILOX" if args.rng != "numpy" else
                 "RNG_NUMPY_DEC" if (kt.get("k_decode") or 0.0) > 0.0 else "RNG_NUMPY_PIPE")
    achieved = launch_steps * ALGO_BYTES_PER_STEP / (play_ms * 1e-3) / 1e9
    dec = play_mode == "RNG_NUMPY_DEC"
    per_kernel, traffic_src = (pmc_traffic(args.rng if dec or args.rng != "numpy" else "numpy_ring", B)
                               if not args.no_obs else (None, None))
    traffic = per_kernel.get("k_play<4") if per_kernel else None
    # bytes the counters saw per launch / its duration: below `frac` when the
    # game state stays in VGPRs within a launch (SURVEY §8(d) counts it twice)
    real_frac = traffic / (play_ms * 1e-3) / 1e9 / HBM_PEAK_GBS if traffic else None
    result = {
        "metric": "env-steps/sec at 65536 concurrent 4-player games, 1/2/4/8 MI355X",
        "value": value,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3,
        "timed_region_s": wall,
        "host_enqueue_ms_per_step": ENQUEUE_S / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (seeded deals: game g = np.random.seed(g) stream)",
        "config": {
            "workload": "config2: 65536 x 4-player DrunkHamster self-play per GPU, one episode (10 env-steps) per "
                        "launch, numpy-MT RNG, int8 obs + actions + rewards + done emitted",
            "games_per_gpu": B,
            "players": N_PLAYERS,
            "env_steps_per_launch": launch_steps,
            "rng": args.rng,
            "obs": not args.no_obs,
            "parallelism": f"dp{world} (independent game shards, no data-path collective)",
            "launches_per_call": args.launches_per_call,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_unit": "HBM bytes per k_play launch (PMC FETCH_SIZE x2 + WRITE_SIZE, separate passes)",
            "traffic_source": traffic_src,
            "real_frac": real_frac,
            "kernel": f"k_play<4, {play_mode}>: 10 env-steps of 65536 games",
            "kernel_ms": play_ms,
            "kernel_ms_source": ("HIP events around each k_play launch on its stream (sn_kernel_times), over a second "
                                 "pass of the same launches right after the timed one" if args.rng == "numpy" else
                                 "HIP events around each timed launch on the launch stream"),
            "algo_bytes_per_env_step": ALGO_BYTES_PER_STEP,
            "algo_bytes_per_launch": launch_steps * ALGO_BYTES_PER_STEP,
            "step_ms": kern_ms,
            "step_frac": launch_steps * ALGO_BYTES_PER_STEP / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "concurrent": ({"kernel": "k_mt_ahead<false, true> (side stream: one dispatch per twist_every play "
                                      "launches, whole MT19937 rounds ahead of the consumer)",
                            "kernel_ms": kt.get("k_mt_ahead"),
                            "decode_kernel": "k_decode<4> (second side stream, concurrent with the group's twist: "
                                             "the next group's episode records -- draws, deals, stream offsets -- "
                                             "for k_play<4, RNG_NUMPY_DEC>; SN_OPT_PIPE_DEC)",
                            "decode_kernel_ms": kt.get("k_decode"),
                            "decode_traffic": per_kernel.get("k_decode") if per_kernel else None,
                            "decode_dispatches_per_play_launch": (per_kernel["_ratio"].get("k_decode")
                                                                  if per_kernel else None),
                            "traffic": per_kernel.get("k_mt_ahead<false") if per_kernel else None,
                            "traffic_unit": "HBM bytes per steady twist dispatch (PMC)",
                            "twist_dispatches_per_play_launch": (per_kernel["_ratio"].get("k_mt_ahead<false")
                                                                 if per_kernel else None)}
                           if args.rng == "numpy" else None),
            # sum over the step's kernels of PMC bytes per dispatch x measured dispatches per play launch
            # (the traffic file's own counts: recomputable by hand from it)
            "step_traffic": per_kernel.get("_step") if per_kernel else None,
            "twist_every": twist_k if args.rng == "numpy" else None,
        },
        "episodes_checksum": {"episodes": int(eps.sum().item()) * world, "mean_score_per_seat": (tot / (eps.sum().item() * world)).tolist()},
    }
    if rank == 0 and world == 1 and not args.no_cpu and want("cpu"):
        result["cpu_baseline"] = cpu_baseline(args.cpu_seconds, args.rng)
    if world == 1 and not args.no_mcs and want("mcs"):
        result["extra_config3_mcs"] = bench_mcs(args.mcs_games, args.mcs_rollouts)
    if world == 1 and not args.no_puct and want("puct"):
        result["extra_config4_puct"] = bench_puct(args.puct_games)
        result["extra_config4_customed"] = bench_customed(args.puct_games)
        result["extra_acer"] = bench_acer(args.puct_games // 2)
    if world == 1 and not args.no_scalar and want("scalar"):
        result["extra_config1_scalar"] = bench_scalar()
    if not args.no_league and want("league"):
        league = bench_league(world, rank, B, args.league_rounds)
        if rank == 0:
            result["extra_config5_tournament"] = league
    if not args.no_mixed_league and want("mixed"):
        mixed = bench_league_mixed(world, rank, args.mixed_slots, args.mixed_mc_max)
        if rank == 0:
            result["extra_config5_run_py_league"] = mixed
    if world == 1 and not args.no_dropin and want("dropin"):
        result["extra_dropin_search"] = bench_dropin()
    if world == 1 and not args.no_philox and args.rng == "numpy" and want("philox"):
        # config 2 in the counter-based mode ("philox ... used for
        # throughput"): same games-per-launch, role-split k_play (SN_OPT_PLAY_SPLIT 1)
        env2 = VecSechsNimmtEnv(B, N_PLAYERS, seed=0, rng="philox")
        env2.reset()
        w2, k2, _ = time_rollouts(env2, out, args.steps, args.warmup, world)
        env2.close()
        ach2 = launch_steps * ALGO_BYTES_PER_STEP / (k2 * 1e-3) / 1e9
        pk2, src2 = pmc_traffic("philox", B)
        tr2 = pk2.get("k_play_split<4") if pk2 else None
        result["extra_config2_philox"] = {
            "metric": "env-steps/sec at 65536 concurrent 4-player games (philox RNG mode)",
            "value": B * STEPS_PER_LAUNCH * args.steps / w2, "unit": "env-steps/s",
            "ms_per_step": w2 / args.steps * 1e3,
            "roofline": {"bound": "hbm", "achieved": ach2, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": ach2 / HBM_PEAK_GBS, "traffic": tr2, "traffic_source": src2,
                         "real_frac": tr2 / (k2 * 1e-3) / 1e9 / HBM_PEAK_GBS if tr2 else None,
                         "kernel": "k_play_split<4, RNG_PHILOX>: producer waves decode the draws into LDS",
                         "kernel_ms": k2, "kernel_ms_source": "HIP events around each timed launch on the launch stream"},
        }
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
