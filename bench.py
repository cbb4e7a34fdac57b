#!/usr/bin/env python3
"""bench.py — decided+applied instances/s for the MI355X batched-consensus engine.

Workload (BASELINE.json configs[4], SURVEY §8(d) config 5, per GPU): 65,536 independent Paxos
groups x 256 instances x 4 AcceptReplies (N = 5) + 4 PUT/GET commands per instance, per-group
keys uniform on [0,256). One step = for every group: the accept tally (handleAcceptReply, MIN
by default), executeCommands over the committed prefix against the group's KV table, the step
totals (instances decided / executed, commands executed), then ONE RCCL group per step: max of
the commit/executed watermark vector of all groups of the job and sum of the totals, issued on a
second HIP stream so it overlaps the next step's kernel (double-buffered watermark vectors).
  --scaling weak    each rank owns --groups groups (default)
  --scaling strong  --groups-total groups split over the ranks (block partition)
`value` = instances DECIDED by the step (quorum crossings, summed over ranks by the step's
all-reduce) per second; every one of them is also executed in the same step (MIN executes up to
committedUpTo, the highest decided instance). Executed instances / commands per second are
reported beside it.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--mode min|classic]
  torchrun --nproc-per-node N bench.py --gpus N ...

`--gpus N` (N > 1) without a launcher (no WORLD_SIZE in the environment) starts N fresh rank
processes itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT), before
anything loads the engine or touches a GPU, waits for all of them, forwards rank 0's JSON line
and exits non-zero if any rank fails. Under torchrun the ranks come from the environment.
The default is BASELINE config 5 as written: 65,536 groups in total, strong scaling (block
partition over the ranks); `--scaling weak --groups G` keeps G groups per GPU instead.

The other single-GPU configurations of BASELINE.json are kernel benches of their own
(--workload; the default `step` is the headline line above):
  tally       config 2: accept tally, 16M instances x 4 replies (k_accept_tally), --mode min|classic
  prepare     config 3: CLASSIC prepare selection, 16M instances x 4 replies (k_prepare_classic)
  prepare_min config 3, MIN variant: one PrepareBookkeeping per group, G = 65,536 (k_prepare_min)
  apply       config 4: batched KV apply, 64M PUT/GET over 1M keys (mpx_apply), --dist uniform|zipf
  conflict    state.ConflictBatch of consecutive instances of the config-4 commands, B = 4
  decode      SURVEY §8(f) rank 1: peer-stream framing + AcceptReply decode of the config-2 replies
              (fixed-size frames; stops at the first variable-length message)
  stream      SURVEY §8(f) rank 1, full: a leader's stream with PrepareReplies mixed in
              (--mode min|classic wire, --prepare-every K, --prep-cmds n), every frame decoded
  fanout      SURVEY §8(f) rank 2: ProposeReplyTS fan-out of 64M replies over --clients connections
  log         SURVEY §8(f) ranks 3/4: instance-log encoding of 16M committed instances x 4 commands
  replay      SURVEY §8(f) rank 3 (read side): durable-log replay of 16M 29-byte records
Each prints one JSON line in the same format, with its own roofline, parity and CPU baseline.

Device memory, streams and events come from the engine's own HIP runtime (mpx_dev_alloc & co):
libmpx.so is loaded before anything imports torch, so it binds /opt/rocm's HIP and RCCL — the
runtime the tests run on, recorded in the line's "runtime" field. torch is only imported for the
gloo group (unique-id broadcast, barriers, max over ranks) when WORLD_SIZE > 1. Inputs are
generated on the host (counter-based splitmix64) and copied to HBM before timing; the timed
region contains only device work.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# _lib.load() runs in main(), after the rank launcher and before torch is imported (the engine's
# HIP + RCCL, not torch's); importing this module loads nothing
from minpaxos_amd import _lib  # noqa: E402
from minpaxos_amd import records as R  # noqa: E402
from minpaxos_amd import shard, synth  # noqa: E402
from minpaxos_amd.devbuf import D2D, Arena, DevArray  # noqa: E402
from minpaxos_amd.engine import Engine, MpxError, step_one_launch_fits  # noqa: E402

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mode", default="min", choices=["min", "classic"])
    ap.add_argument("--scaling", default="strong", choices=["weak", "strong"],
                    help="strong (default): --groups-total split over the ranks (BASELINE "
                         "config 5); weak: --groups per rank")
    ap.add_argument("--groups", type=int, default=8192,
                    help="groups per GPU (weak scaling; SURVEY 8(d): 8192 per GPU)")
    ap.add_argument("--groups-total", type=int, default=65536,
                    help="groups of the whole job (strong scaling)")
    ap.add_argument("--ipg", type=int, default=256)
    ap.add_argument("--cmds", type=int, default=4)
    ap.add_argument("--keys", type=int, default=256)
    ap.add_argument("--replicas", type=int, default=5, help="N (replies per instance = N-1)")
    ap.add_argument("--kv-per-group", type=int, default=256,
                    help="group table capacity (config 5: the per-group key space, 256)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="issue the step all-reduce on the compute stream (no overlap)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-groups", type=int, default=0,
                    help="groups timed on the CPU baseline (0 = auto, ~10-30 s of CPU work)")
    ap.add_argument("--parity-groups", type=int, default=512)
    ap.add_argument("--traffic-json", default="")
    ap.add_argument("--workload", default="step",
                    choices=["step", "tally", "prepare", "prepare_min", "apply", "conflict",
                             "decode", "stream", "fanout", "log", "replay"])
    ap.add_argument("--prepare-every", type=int, default=4096,
                    help="stream: a PrepareReply before every K-th AcceptReply (0 = none)")
    ap.add_argument("--prep-cmds", type=int, default=1,
                    help="stream: Commands carried by each PrepareReply")
    ap.add_argument("--log-format", default="catchup", choices=["catchup", "durable"])
    ap.add_argument("--clients", type=int, default=1024, help="fanout: client connections")
    ap.add_argument("--instances", type=int, default=1 << 24, help="tally / prepare: instances")
    ap.add_argument("--prep-groups", type=int, default=65536, help="prepare_min: groups")
    ap.add_argument("--commands", type=int, default=1 << 26, help="apply: commands")
    ap.add_argument("--apply-keys", type=int, default=1 << 20, help="apply: key space")
    ap.add_argument("--kv-capacity", type=int, default=0,
                    help="apply: engine key capacity (0 = --apply-keys; the table gets >= 2x slots, load <= 1/2)")
    ap.add_argument("--dist", default="uniform", choices=["uniform", "zipf"])
    ap.add_argument("--kernel-events", default="separate", choices=["separate", "inline"],
                    help="step, enqueued pass: HIP events around the group kernel in a separate "
                         "pass after the timed steps (default) or inside the timed steps")
    ap.add_argument("--step-launches", type=int, default=2, choices=[1, 2],
                    help="step: 1 = MPX_FLAG_STEP_ONE_LAUNCH (the fast kernel alone, totals "
                         "folded by its last workgroup) where the shape fits a fast variant, "
                         "2 = fast + work-list kernel (the default: 0.097 vs 0.103 ms per "
                         "step at --emulate-world 8, DESIGN §9)")
    ap.add_argument("--separate-totals", action="store_true",
                    help="step: the totals by their own launch after the group step "
                         "(mpx_step_totals_dev) instead of the step's work-list kernel "
                         "(mpx_group_step_totals_dev, the default: two launches per step)")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="step: one process measures the share of ONE rank of a P-rank job (P = "
                         "this value): it owns groups [0, G_total/P) of the job's G_total, the "
                         "watermark vector stays 2 x G_total through the engine's all-reduce "
                         "(one rank: RCCL's copy); a proxy for the per-rank cost of strong / weak "
                         "scaling, not a multi-GPU measurement")
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                    help="step: after the timed loop, capture the step sequence (group step, "
                         "totals, the RCCL group on the second stream, the double-buffer "
                         "event waits) into hipGraphs of up to 64 steps (mpx_graph_*) and time "
                         "their replay; value / ms_per_step then come from the replay. auto = "
                         "on in one process (a one-rank communicator, validated on the GPU "
                         "box), off across processes (RCCL capture across ranks unvalidated)")
    ap.add_argument("--apply-path", default="auto",
                    choices=["auto", "small", "sorted", "partitioned"],
                    help="apply: mpx_config.apply_path (auto = by call size)")
    ap.add_argument("--replay-dups", action="store_true",
                    help="replay: instNo drawn with repeats (last record wins) instead of a permutation")
    ap.add_argument("--replay-atomic", action="store_true",
                    help="replay: no mpx_replay_durable_reserve, so one device atomic per record "
                         "(the A/B of the binned slot maximum)")
    return ap.parse_args()


class Ranks:
    """The process group of a multi-GPU run, for host-side coordination only (gloo on CPU):
    the RCCL unique id broadcast, barriers around the timed region and the max over ranks of
    the elapsed time. Device data moves only through the engine's RCCL communicator."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        if self.world > 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            import torch.distributed as dist
            dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, x):
        if not self.dist:
            return x
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def bcast(self, obj):
        if not self.dist:
            return obj
        box = [obj if self.rank == 0 else None]
        self.dist.broadcast_object_list(box, src=0)
        return box[0]

    def gather(self, obj):
        """obj of every rank, in rank order, on every rank"""
        if not self.dist:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def close(self, barrier=True):
        if self.dist:
            if barrier:
                self.dist.barrier()
                self.dist.destroy_process_group()


def host_cores():
    """the CPU share of this process: its affinity set, capped by OMP_NUM_THREADS (16 on the
    GPU box, whose nproc reports the whole machine) and by 16"""
    n = len(os.sched_getaffinity(0))
    lim = os.environ.get("OMP_NUM_THREADS", "")
    if lim.isdigit() and int(lim) > 0:
        n = min(n, int(lim))
    return max(1, min(n, 16))


TRAFFIC_DB = os.path.join(ROOT, "profiles", "traffic_r06.json")
ISSUE_BOUND = ("decode", "stream", "fanout")


def traffic_for(key, alg, path=""):
    """HBM bytes per launch of the measured call from a committed rocprofv3 counter pass
    (tools/pmc_collect.py: FETCH_SIZE x 2 + WRITE_SIZE, separate --pmc passes, summed over the
    call's kernels) taken on EXACTLY this configuration (`key`: workload and every parameter
    that changes the kernel variant or the bytes moved). Returns (bytes or None, note); a
    figure below the algorithmic bytes cannot be this configuration's and is rejected."""
    try:
        db = json.load(open(path or TRAFFIC_DB))
    except Exception:
        return None, "no counter database"
    for ent in db.get("entries", []):
        if ent.get("key") == key:
            b = ent.get("bytes_per_launch")
            if b is None:
                return None, "no FETCH/WRITE pass for this exact configuration"
            if b < alg:
                return None, f"counter pass ({b:.4g} B) below the algorithmic bytes: rejected"
            return b, ent.get("source", "")
    return None, "no counter pass for this exact configuration"


# issue peaks for the rows bound by instruction issue rather than HBM (MI355X_MICROARCH.md:
# a wave64 VALU instruction issues over 2 cycles on its SIMD; an LDS wave-instruction takes at
# least 2 LDS-array cycles per CU, ds_read_b32/b64 rate), 256 CUs x 4 SIMDs at 2.4 GHz
PEAK_VALU_GIPS = 256 * 4 * 0.5 * 2.4   # G wave-instructions / s
PEAK_LDS_GIPS = 256 * 0.5 * 2.4


def instr_for(key, path=""):
    """SQ instruction counts per launch (tools/pmc_collect.py --instr) of exactly this
    configuration, or None"""
    try:
        db = json.load(open(path or TRAFFIC_DB))
    except Exception:
        return None
    for ent in db.get("entries", []):
        if ent.get("key") == key and ent.get("instr"):
            return ent["instr"]
    return None


def issue_roofline(kernel, key, kern_ms, hbm, path=""):
    """the roofline object of a row not bound by HBM bandwidth: VALU and LDS wave-instructions
    per launch (counter database) against the issue peaks, and the SQ wave-cycle split (parked
    at s_waitcnt / barriers, issue-stalled, issuing: MI355X_MICROARCH.md, the three are disjoint
    and sum to SQ_WAVE_CYCLES). bound = "valu" / "lds" when that issue fraction is at least 0.5,
    else "latency" when parked is the largest of the three shares, "issue-stall" when issue
    stalls are, else "issue (mixed)" (the HBM figures then carry the row: achieved / peak / frac
    are its HBM numbers). Without a counter
    pass the bound stays "valu"  with achieved null."""
    ins = instr_for(key, path) or {}
    t = kern_ms * 1e-3
    valu, lds = ins.get("SQ_INSTS_VALU"), ins.get("SQ_INSTS_LDS")
    fv = valu / t / 1e9 / PEAK_VALU_GIPS if valu else None
    fl = lds / t / 1e9 / PEAK_LDS_GIPS if lds else None
    wc = ins.get("SQ_WAVE_CYCLES")
    waits = {k: ins[k] / wc for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")
             if wc and k in ins}
    # mean resident waves per CU over the call's kernels: SQ_WAVE_CYCLES counts quad-cycles
    # summed over every wave, GRBM_GUI_ACTIVE the busy cycles summed over the 8 XCDs
    # (MI355X_MICROARCH.md), so waves / CU = 4 x WAVE_CYCLES / (GRBM / 8 x 256 CUs)
    grbm = ins.get("GRBM_GUI_ACTIVE")
    if wc and grbm:
        waits["mean_waves_per_cu"] = wc * 4.0 / (grbm / 8.0 * 256)
    use_lds = fl is not None and (fv is None or fl > fv)
    top = max(x for x in (fv, fl, 0.0) if x is not None)
    out = {"kernel": kernel, "valu_frac": fv, "lds_frac": fl,
           "valu_instr_per_launch": valu, "lds_instr_per_launch": lds,
           "wave_cycle_split": waits or None,
           "instr_note": "SQ_INSTS_VALU / SQ_INSTS_LDS and SQ_WAVE_CYCLES / SQ_WAIT_ANY / "
                         "SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY (+ GRBM_GUI_ACTIVE for the mean "
                         "resident waves per CU) rocprofv3 passes "
                         "(tools/pmc_collect.py --instr) of this exact configuration" if ins else
                         "no instruction-counter pass for this exact configuration",
           "hbm": hbm}
    if top >= 0.5 or not waits:
        out.update({"bound": "lds" if use_lds else "valu",
                    "achieved": (lds if use_lds else valu) / t / 1e9 if (valu or lds) else None,
                    "peak": PEAK_LDS_GIPS if use_lds else PEAK_VALU_GIPS,
                    "unit": "G wave-instr/s", "frac": fl if use_lds else fv})
    else:
        wa, wi, ac = (waits.get(k, 0.0) for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                                   "SQ_ACTIVE_INST_ANY"))
        out.update({"bound": "latency" if wa >= max(wi, ac) else
                    "issue-stall" if wi >= ac else "issue (mixed)",
                    "achieved": hbm["achieved"], "peak": hbm["peak"], "unit": hbm["unit"],
                    "frac": hbm["frac"]})
    return out


def launch_ranks(n):
    """--gpus n without a launcher: n fresh child processes of this script, one per GPU. The
    parent never loads the engine or touches a GPU (no HIP call precedes the children); it
    forwards rank 0's stdout, sends the other ranks' stdout to stderr, and ends every rank as
    soon as one fails. Returns the exit status."""
    import socket
    import subprocess
    import threading
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env, stdout=subprocess.PIPE if r == 0 else sys.stderr))

    def forward(pipe):
        for ln in iter(pipe.readline, b""):
            sys.stdout.write(ln.decode(errors="replace"))
            sys.stdout.flush()
    fw = threading.Thread(target=forward, args=(procs[0].stdout,), daemon=True)
    fw.start()
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c
                print(f"bench.py: rank {procs.index(p)} exited with status {c}; stopping the "
                      f"other ranks", file=sys.stderr, flush=True)
                for q in live:
                    q.kill()  # the exact child PIDs this parent started
        time.sleep(0.05)
    fw.join(timeout=10)
    return rc


# ==================================== headline: config 5 ======================================
def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a.gpus))
    _lib.load()
    rk = Ranks()
    if a.gpus != rk.world and rk.rank == 0:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={rk.world}; running {rk.world} ranks",
              file=sys.stderr, flush=True)
    ok = False
    try:
        if a.workload == "step":
            step_bench(a, rk)
        else:
            kernel_bench(a, rk)
        ok = True
    finally:
        # a failed rank leaves without the closing barrier (its peers may be blocked in another
        # collective): it exits non-zero and the launcher ends the others
        rk.close(barrier=ok)


def step_bench(a, rk):
    world, rank = rk.world, rk.rank
    mode = R.MODE_MIN if a.mode == "min" else R.MODE_CLASSIC
    N, ipg, B, K = a.replicas, a.ipg, a.cmds, a.kv_per_group
    emu = a.emulate_world
    if emu and world != 1:
        raise SystemExit("--emulate-world runs in one process (it measures one rank's share)")
    P = emu or world  # ranks of the job whose per-rank share this process runs
    if a.scaling == "weak":
        G_total = a.groups * P
    else:
        G_total = a.groups_total
    g0, g1 = shard.block_range(G_total, P, rank)
    G = g1 - g0
    one_launch = a.step_launches == 1 and step_one_launch_fits(N, ipg, K) and not a.separate_totals
    eng = Engine(rk.local, n_replicas=N, mode=mode, kv_per_group=K, max_groups=max(G, 1),
                 step_one_launch=one_launch)
    ar = Arena(eng)

    # ---- this rank's block of groups, generated from their global ids --------------------------
    t_gen = time.time()
    b = synth.group_batch(G, ipg, N, B, a.keys, p_ok=0.7, p_put=0.5, seed=45, first_group=g0)
    t_gen = time.time() - t_gen
    m = len(b["op"])
    d = dict(
        recs=ar.put(b["recs"]), off=ar.put(b["grp_rec_off"]), st_in=ar.put(b["st_in"]),
        st_out=ar.put(b["st_in"]),  # instances without replies keep their input state
        ci=ar.put(b["committed_in"]), ei=ar.put(b["executed_in"]), pi=ar.put(b["peer_in"]),
        po=ar.empty(G * N, np.int32), op=ar.put(b["op"]), key=ar.put(b["key"]),
        val=ar.put(b["val"]), coff=ar.put(b["cmd_off"]),
        ret=ar.full(m, np.int64, 0), conf=ar.full(m, np.uint8, 0),
        kc0=ar.full(G, np.uint32, 0), kk0=ar.full(G * K, np.int64, 0),
        kv0=ar.full(G * K, np.int64, 0), kc1=ar.full(G, np.uint32, 0),
        kk1=ar.full(G * K, np.int64, 0), kv1=ar.full(G * K, np.int64, 0),
        nd=ar.full(G, np.uint32, 0),
        # the step's watermark vectors, double-buffered: the group step writes this rank's
        # groups into a send vector whose other ranges hold -1 for good (filled once below;
        # the buffers start poisoned, 0x7F7F7F7F > any instance, so a missing fill or a group
        # the step skipped shows up), the max over ranks lands in the receive vector
        wms=[ar.full(2 * G_total, np.int32, 0x7F) for _ in range(2)],
        wmr=[ar.full(2 * G_total, np.int32, 0x7F) for _ in range(2)],
        tot=[ar.full(R_TOTALS, np.int64, 0) for _ in range(2)],
    )

    def batch(buf, tin, tout):
        wm = d["wms"][buf]
        kc_i, kk_i, kv_i = tin
        kc_o, kk_o, kv_o = tout
        return _lib.MpxGroupBatch(
            G, ipg, d["recs"].ptr, d["off"].ptr, d["st_in"].ptr, d["st_out"].ptr, d["ci"].ptr,
            wm.at(g0), d["ei"].ptr, wm.at(G_total + g0), d["pi"].ptr, d["po"].ptr, d["op"].ptr,
            d["key"].ptr, d["val"].ptr, d["coff"].ptr, None, d["ret"].ptr, d["conf"].ptr,
            kc_i.ptr, kk_i.ptr, kv_i.ptr, kc_o.ptr, kk_o.ptr, kv_o.ptr, None, d["nd"].ptr)

    t0s = (d["kc0"], d["kk0"], d["kv0"])
    t1s = (d["kc1"], d["kk1"], d["kv1"])
    comp = eng.stream
    comm = comp if a.no_overlap else eng.stream_create()
    uid = rk.bcast(Engine.comm_unique_id() if rank == 0 else None)
    eng.comm_init(world, rank, uid)

    # steady state: the group tables already hold their keys (one untimed step fills them),
    # and every timed step reads that table and writes a fresh one (same work every step)
    eng.group_step_dev(batch(0, t1s, t0s), comp)
    eng.synchronize()
    steps = [batch(0, t0s, t1s), batch(1, t0s, t1s)]
    ev_done = [eng.event_create(False) for _ in range(2)]
    ev_comm = [eng.event_create(False) for _ in range(2)]
    n_ev = max(a.steps, 1)
    ev_k = [(eng.event_create(), eng.event_create()) for _ in range(n_ev)]

    # watermark ranges other ranks own, [0, g0) and [g1, G_total) of both halves: -1 once
    for lo, hi in [(h + lo, h + hi) for h in (0, G_total) for lo, hi in ((0, g0), (g1, G_total))
                   if hi > lo]:
        for wb in d["wms"]:
            eng.memset(wb.at(lo), 0xFF, (hi - lo) * 4, comp)
    eng.synchronize()

    def step(i, timed, evs=None, cs=None):
        cs = cs or comm  # the collective's stream
        buf = i & 1
        if i >= 2:  # buffers `buf` are free once the all-reduce of step i-2 has used them
            eng.stream_wait_event(comp, ev_comm[buf])
        # the timed steps' HIP events bracket the group kernel alone: the engine records them
        # right before and after its launch (mpx_group_step_events), the work-list kernel and
        # the totals are outside. Steps without events make no hook call at all (the hook is
        # off between evented steps), so the enqueued timed loop carries no extra ctypes calls
        use_ev = evs or (ev_k[i] if timed else None)
        if use_ev:
            eng.group_step_events(*use_ev)
        # the group step, then its totals (decided, executed instances, executed commands)
        if not a.separate_totals:
            eng.group_step_totals_dev(steps[buf], d["tot"][buf].ptr, comp)
        else:
            eng.group_step_dev(steps[buf], comp)
        if use_ev:
            eng.group_step_events()
        if a.separate_totals:
            eng.step_totals_dev(steps[buf], d["tot"][buf].ptr, comp)
        eng.event_record(ev_done[buf], comp)
        eng.stream_wait_event(cs, ev_done[buf])
        eng.step_allreduce_oop_dev(d["wms"][buf].ptr, d["wmr"][buf].ptr, G_total,
                                   d["tot"][buf].ptr, R_TOTALS, cs)
        eng.event_record(ev_comm[buf], cs)

    use_graph = a.graph == "on" or (a.graph == "auto" and world == 1)
    for i in range(a.warmup):
        step(i, False)
    eng.synchronize()
    rk.barrier()
    eng.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(i, a.kernel_events == "inline")
    t_enq = time.perf_counter() - t0  # host time to enqueue the timed steps
    eng.synchronize()  # every stream of the device; raises if a kernel flagged an error
    rk.barrier()
    t1 = time.perf_counter()
    elapsed = rk.max(t1 - t0)
    n_kev = 0
    if a.kernel_events == "inline":
        kern_ms = [eng.event_elapsed_ms(e0, e1) for e0, e1 in ev_k[:a.steps]]
    else:
        # the kernel times from a separate pass of the same steps right after the timed region:
        # timing events between the kernels of every timed step cost the enqueued step ~17 us
        # (a timestamp write on the compute stream per event; --emulate-world 8: 0.117-0.120 ms
        # per step with them), so the timed steps carry none
        n_kev = min(a.steps, n_ev, 64)
        for j in range(n_kev):
            step(a.steps + j, True, ev_k[j])
        eng.synchronize()
        rk.barrier()
        kern_ms = [eng.event_elapsed_ms(e0, e1) for e0, e1 in ev_k[:n_kev]]
    last = (a.steps + n_kev - 1) & 1
    graph_info = None
    if use_graph:
        # the same step sequence replayed from hipGraphs, a chunk of U steps per capture. The
        # graph runs the collective on the compute stream: a replayed graph executed the
        # second stream's copy and its event edges between a step's kernels and the next step's
        # anyway (profiles/r05/step), and one stream leaves out two cross-stream dependencies
        # per step (--emulate-world 8: 0.113 -> 0.097 ms per step). The graph pass is one
        # process: the one-rank all-reduce is RCCL's copy.
        U = min(a.steps, 64)
        chunks = [U] * (a.steps // U) + ([a.steps % U] if a.steps % U else [])
        # a second U-step graph, the same steps with a HIP event pair around each group kernel
        # (external event nodes, which cost a replay a few us per step, so the timed graphs have
        # none): replayed once after the timed region, it gives the roofline's kernel times
        ev_g = [(eng.event_create(), eng.event_create()) for _ in range(U)]

        def capture(n, evs=False):
            eng.graph_begin(comp)
            for j in range(n):
                step(j, False, ev_g[j] if evs else None, cs=comp)
            return eng.graph_end(comp)
        g_ev = None
        try:
            graphs = {n: capture(n) for n in set(chunks)}
        except MpxError as e:  # "auto" on a library without stream capture (the CPU stub)
            if a.graph == "on":
                raise
            graph_info = {"used": False, "unavailable": str(e)[:160]}
            use_graph = False
        if use_graph:
            try:
                g_ev = capture(U, evs=True)
            except MpxError:  # (a runtime without external event nodes: the enqueued pass's)
                g_ev = None
    if use_graph:
        for _ in range(max(a.warmup, 1)):
            eng.graph_launch(graphs[U], comp)
        eng.synchronize()
        rk.barrier()
        eng.synchronize()
        t0 = time.perf_counter()
        for n in chunks:
            eng.graph_launch(graphs[n], comp)
        eng.synchronize()
        rk.barrier()
        t1 = time.perf_counter()
        elapsed_graph = rk.max(t1 - t0)
        graph_info = {"used": True, "steps_per_graph": U, "graph_launches": len(chunks),
                      "collective_stream": "compute (in the graph)",
                      "ms_per_step_graph": elapsed_graph / a.steps * 1e3,
                      "ms_per_step_no_graph": elapsed / a.steps * 1e3,
                      "kernel_ms_median_enqueued": float(np.median(kern_ms))}
        if g_ev is not None:
            for _ in range(3):  # (the first replays of a fresh graph run cold)
                eng.graph_launch(g_ev, comp)
            eng.synchronize()
            kern_ms = [eng.event_elapsed_ms(e0, e1) for e0, e1 in ev_g]
            graph_info["kernel_times"] = ("the third replay of the timed graph's steps with an "
                                          "event pair around each group kernel")
            graph_info["evented_replay_steps"] = 3 * U
            eng.graph_destroy(g_ev)
        else:
            graph_info["kernel_times"] = "the enqueued pass's events"
        last = ((U if g_ev is not None else chunks[-1]) - 1) & 1  # the last replayed step
        elapsed = elapsed_graph
        for gx in graphs.values():
            eng.graph_destroy(gx)

    # ---- outputs of the (identical) timed steps -------------------------------------------------
    tot = ar.get(d["tot"][last])  # summed over ranks by the step's all-reduce
    n_decided, n_exec_inst, n_exec_cmds = (int(x) for x in tot)
    wm = ar.get(d["wmr"][last])
    committed, executed = wm[:G_total], wm[G_total:]
    own_e = executed[g0:g1].astype(np.int64)
    kc = ar.get(d["kc1"])
    # every rank sees every group's watermark (no -1 or poison left) and all ranks hold the
    # same vector after the all-reduce; an emulated rank holds its own range and -1 elsewhere
    if emu:
        foreign = np.ones(G_total, bool)
        foreign[g0:g1] = False
        wm_ok = bool((committed[g0:g1] >= 0).all() and (executed[g0:g1] < ipg).all()
                     and (committed[g0:g1] < ipg).all() and (committed[foreign] == -1).all()
                     and (executed[foreign] == -1).all())
    else:
        wm_ok = bool((committed >= 0).all() and (wm < ipg).all())
    import hashlib
    wm_sha = hashlib.sha256(wm.tobytes()).hexdigest()
    shas = rk.gather(wm_sha)
    coff = b["cmd_off"].astype(np.int64)
    gidx = np.arange(G, dtype=np.int64) * ipg
    own_cmds = int((coff[gidx + own_e + 1] - coff[gidx]).sum())

    # algorithmic bytes of one group-step launch (this rank): replies + instance state in/out,
    # executed commands (op,key,val in; ret,conf out), group table in/out, per-group scalars
    n_rec = len(b["recs"])
    alg = (n_rec * 16 + G * ipg * 16 * 2 + own_cmds * (17 + 9)
           + int(kc.sum()) * 16 * 2 + G * (4 * 4 + 2 * N * 4 + 4 * 2 + 8 * 2 + 4))
    kern_avg_ms = float(np.mean(kern_ms)) if kern_ms else float("nan")
    kern_med_ms = float(np.median(kern_ms)) if kern_ms else float("nan")
    # the kernel's time is bounded from above by its event bracket (the kernel plus the dispatch
    # on either side and the event nodes' own cost) and by the step it is part of (the kernel
    # plus the work-list kernel and the collective): achieved from the tighter bound, so the
    # kernel is never credited with more time than the step took (the bracket came out 0.2 %
    # above ms_per_step on one box)
    step_ms = elapsed / max(a.steps, 1) * 1e3
    kern_bound_ms = min(kern_avg_ms, step_ms)
    achieved_gbs = alg / (kern_bound_ms * 1e-3) / 1e9
    tkey = {"workload": "step", "mode": a.mode, "groups": G, "ipg": ipg, "replicas": N,
            "cmds": B, "keys": a.keys, "kv_per_group": K}
    traffic, tnote = traffic_for(tkey, alg, a.traffic_json)

    res = {}
    if rank == 0:
        # parity: the first groups of the timed output against the oracle (test infra)
        res["parity"] = parity_sample(b, d, ar, a, mode, N, K, G_total, g0, last)
        if world == 1 and not a.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(b, a, mode, N, K)

    if rank == 0:
        cfg_work = (f"config5: {G_total} groups ({a.scaling} scaling, {G} on rank 0) x {ipg} "
                    f"instances x {N - 1} AcceptReplies + {B} cmds/instance, keys U[0,{a.keys}) "
                    f"per group, mode {a.mode}")
        if emu:
            cfg_work += (f"; EMULATED rank 0 of {emu}: one process, groups [{g0}, {g1}) of "
                         f"{G_total}, the full {2 * G_total}-entry watermark vector through a "
                         f"one-rank RCCL all-reduce")
        line = {
            "metric": "decided+applied instances/sec (tally + KV apply + RCCL watermark all-reduce)",
            "value": n_decided * a.steps / elapsed,
            "unit": "instances/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": a.scaling,
            "vs_baseline": None,
            "dtype": "int32/int64",
            "data": "synthetic (counter-based splitmix64, SURVEY §8(d) config 5)",
            "config": {
                "workload": cfg_work,
                "groups_total": G_total, "groups_per_rank": G, "instances_per_step": G_total * ipg,
                "commands_per_step": G_total * ipg * B, "parallelism": f"groups block-sharded x{world}",
                "collective": ("one RCCL group per step: out-of-place all-reduce(max) of 2 x "
                               "groups_total int32 watermarks + all-reduce(sum) of 3 int64 step "
                               "totals, "
                               + ("on the compute stream" if a.no_overlap or use_graph else
                                  "on a second stream overlapping the next step's kernel")),
            },
            "value_counts": "instances decided by the step (quorum crossings), all ranks",
            "roofline": {
                "bound": "hbm", "kernel": "k_group_fast", "achieved": achieved_gbs,
                "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": achieved_gbs / PEAK_HBM_GBS,
                "traffic": traffic, "traffic_note": tnote, "traffic_key": tkey,
                "traffic_kernels": ["k_group_fast"],
                "alg_bytes_per_launch": alg,
                "alg_table_bytes": int(kc.sum()) * 16 * 2,
                "alg_note": ("replies 16 B + instance state 16 B in + 16 B out, executed commands "
                             "17 B in + 9 B out, per-group scalars, and the group KV tables 16 B "
                             "per live key in + out (the step re-reads its unchanged table: "
                             "alg_table_bytes of the total)"),
                "kernel_ms_avg": kern_avg_ms, "kernel_ms_median": kern_med_ms,
                "kernel_ms_min": float(np.min(kern_ms)),
                "kernel_ms_bound": kern_bound_ms,
                "frac_at_median": alg / (min(kern_med_ms, step_ms) * 1e-3) / 1e9 / PEAK_HBM_GBS,
                "timing": ("HIP events recorded by the engine right before and after each "
                           "k_group_fast launch (mpx_group_step_events) on the compute stream - "
                           "in a replay of the timed hipGraph (external event nodes) when the "
                           "line is the graph pass, as ms_per_step is, else in an enqueued pass "
                           "of the same steps right after the timed region (--kernel-events); "
                           + ("one launch per step: the kernel's last workgroup folds the step "
                              "totals inside the bracket" if one_launch else
                              "the work-list kernel (second launch) is outside")
                           + "; the collective is outside; achieved from kernel_ms_bound = "
                           "min(their mean, ms_per_step) - both bound the kernel's time from "
                           "above - the median beside it (SURVEY 8(d))"),
                "launches_per_step": 1 if one_launch else 2,
            },
            "enqueue_ms_per_step": t_enq / max(a.steps, 1) * 1e3,  # the enqueued pass's host time
            "decided_instances_per_step": n_decided,
            "executed_instances_per_step": n_exec_inst,
            "executed_commands_per_step": n_exec_cmds,
            "instances_processed_per_s": G_total * ipg * a.steps / elapsed,
            "executed_instances_per_s": n_exec_inst * a.steps / elapsed,
            "executed_commands_per_s": n_exec_cmds * a.steps / elapsed,
            # table fill + warm-up + timed (+ the graph replays' warm-up and timed steps)
            "launches_in_process": 1 + a.warmup + a.steps + n_kev + (
                max(a.warmup, 1) * graph_info["steps_per_graph"] + a.steps
                + graph_info.get("evented_replay_steps", 0) if use_graph else 0),
            "graph": graph_info or {"used": False},
            "watermark_allreduce_ok": wm_ok,
            **({"emulated_world": {
                "ranks": emu, "groups_on_this_rank": G, "groups_total": G_total,
                "per_rank_value": n_decided * a.steps / elapsed,
                "projected_job_value": n_decided * a.steps / elapsed * emu,
                "note": ("one process runs rank 0's share of a P-rank job; projected_job_value "
                         "= P x the per-rank rate, assuming every rank runs as fast and the "
                         "overlapped all-reduce over xGMI stays hidden: a proxy, not a "
                         "multi-GPU measurement")}} if emu else {}),
            "watermarks_sha256": wm_sha,
            "watermarks_identical_on_all_ranks": len(set(shas)) == 1,
            "gen_s": round(t_gen, 2),
            "runtime": _lib.runtime_info(),
        }
        line.update(res)
        print(json.dumps(line), flush=True)
    if comm != comp:
        eng.stream_destroy(comm)
    ar.close()
    eng.close()


R_TOTALS = 3  # mpx_step_totals_dev: decided instances, executed instances, executed commands


def _oracle_sub(b, g0, g1, ipg, N):
    r0, r1 = int(b["grp_rec_off"][g0]), int(b["grp_rec_off"][g1])
    c0, c1 = int(b["cmd_off"][g0 * ipg]), int(b["cmd_off"][g1 * ipg])
    sub = dict(n_groups=g1 - g0, ipg=ipg, recs=b["recs"][r0:r1],
               grp_rec_off=(b["grp_rec_off"][g0:g1 + 1] - np.uint64(r0)),
               st_in=b["st_in"][g0 * ipg:g1 * ipg], committed_in=b["committed_in"][g0:g1],
               executed_in=b["executed_in"][g0:g1], peer_in=b["peer_in"][g0 * N:g1 * N],
               op=b["op"][c0:c1], key=b["key"][c0:c1], val=b["val"][c0:c1],
               cmd_off=(b["cmd_off"][g0 * ipg:g1 * ipg + 1] - np.uint32(c0)))
    return sub, (c0, c1)


def parity_sample(b, d, ar, a, mode, N, K, G_total, g0, last):
    """every output of the first --parity-groups groups of the last timed step against the
    oracle: instance states, decided counts, watermarks (after the all-reduce), peerCommits,
    Execute results, conflicts and the group tables (count, keys, values)"""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import Oracle  # CPU oracle: the checker, never the measured path
    S = min(a.parity_groups, len(b["committed_in"]))
    ipg = a.ipg
    sub, (c0, c1) = _oracle_sub(b, 0, S, ipg, N)
    o = Oracle(N, mode, kv_per_group=K)
    # the timed steps started from the table the warm-up step produced
    w0 = o.group_step(sub)
    want = o.group_step(sub, w0["kv_cnt"], w0["kv_key"], w0["kv_val"])
    wm = ar.get(d["wmr"][last])
    kc = ar.get(d["kc1"], S).astype(np.uint32)
    kk = ar.get(d["kk1"], S * K)
    kv = ar.get(d["kv1"], S * K)
    checks = {
        "st_out": np.array_equal(ar.get(_as(d["st_out"], np.int32), S * ipg * 4),
                                 want["st_out"].view(np.int32).reshape(-1)),
        "n_decided": np.array_equal(ar.get(d["nd"], S), want["n_decided"]),
        "committed": np.array_equal(wm[g0:g0 + S], want["committed_out"]),
        "executed": np.array_equal(wm[G_total + g0:G_total + g0 + S], want["executed_out"]),
        "peer_commits": np.array_equal(ar.get(d["po"], S * N), want["peer_out"]),
        "ret": np.array_equal(ar.get(d["ret"], c1 - c0, c0), want["ret"]),
        "conf_prev": np.array_equal(ar.get(d["conf"], c1 - c0, c0), want["conf_prev"]),
        "kv_cnt": np.array_equal(kc, want["kv_cnt"]),
    }
    tab = True
    for g in range(S):
        n = int(want["kv_cnt"][g])
        tab &= np.array_equal(kk[g * K:g * K + n], want["kv_key"][g * K:g * K + n])
        tab &= np.array_equal(kv[g * K:g * K + n], want["kv_val"][g * K:g * K + n])
    checks["kv_key_val"] = bool(tab)
    bad = [k for k, v in checks.items() if not v]
    return {"groups_checked": S, "outputs": sorted(checks), "bit_exact": not bad,
            "mismatch": bad}


def _as(x, dtype):
    """the same device buffer viewed with another element type"""
    return DevArray(x.ptr, x.nbytes, dtype, (x.nbytes // np.dtype(dtype).itemsize,))


def cpu_baseline(b, a, mode, N, K):
    """the reference-faithful CPU loop (oracle/baseline.cpp), one core, bounded sample"""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as OL
    lib = OL.load()
    ipg = a.ipg
    G = len(b["committed_in"])

    built = {}  # g_n -> (arrays kept alive, batch struct): inputs are never written

    def run(g_n, threads):
        if g_n in built:
            return lib.orc_bench_group_step(N, mode, C.byref(built[g_n][1]), K, threads) * 1e-9
        sub, _ = _oracle_sub(b, 0, g_n, ipg, N)
        o = OL.Oracle(N, mode, kv_per_group=K)
        warm = o.group_step(sub)  # steady-state tables, as on the GPU
        m = len(sub["op"])
        arrs = [g_n, ipg, sub["recs"], sub["grp_rec_off"], sub["st_in"], sub["st_in"].copy(),
                sub["committed_in"], np.zeros(g_n, np.int32), sub["executed_in"],
                np.zeros(g_n, np.int32), sub["peer_in"], np.zeros(g_n * N, np.int32), sub["op"],
                sub["key"], sub["val"], sub["cmd_off"], None, np.zeros(m, np.int64), None,
                warm["kv_cnt"], warm["kv_key"], warm["kv_val"], warm["kv_cnt"].copy(),
                warm["kv_key"].copy(), warm["kv_val"].copy(), None, None]
        arrs = [np.ascontiguousarray(x) if isinstance(x, np.ndarray) else x for x in arrs]
        gb = OL.group_batch_struct(arrs)
        built[g_n] = (arrs, gb)
        ns = lib.orc_bench_group_step(N, mode, C.byref(gb), K, threads)
        return ns * 1e-9

    if a.cpu_sample_groups:
        g_n = min(a.cpu_sample_groups, G)
    else:
        t = run(min(2048, G), 1)
        per = t / min(2048, G)
        g_n = int(min(G, max(2048, 15.0 / max(per, 1e-9))))
    secs, reps = 0.0, 0
    while secs < 10.0 and reps < 50:  # about 10 s of CPU work in total
        secs += run(g_n, 1)
        reps += 1
    out = {"value": g_n * ipg * reps / secs, "unit": "instances/s", "cores": 1, "kind": "port",
           "sample": f"first {g_n} groups of the same workload ({g_n * ipg} instances, "
                     f"{g_n * ipg * (N - 1)} replies, {g_n * ipg * a.cmds} commands) x {reps} "
                     f"reps, pointer-per-instance log + hash-map State, one thread, "
                     f"{secs:.1f} s timed (instances processed per second)"}
    # the same loop with the groups sharded over the process's CPU share (its
    # affinity set, capped by OMP_NUM_THREADS and 16), beside the one-core reference-faithful
    # figure
    th = host_cores()
    if th > 1:
        g_s = min(G, g_n * th)
        ssecs, sreps = 0.0, 0
        while ssecs < 4.0 and sreps < 5:  # each rep also rebuilds the per-group maps (untimed)
            ssecs += run(g_s, th)
            sreps += 1
        out["sharded"] = {"value": g_s * ipg * sreps / ssecs, "unit": "instances/s",
                          "cores": th, "cores_probe": "len(os.sched_getaffinity(0)) capped by "
                                                      "OMP_NUM_THREADS and 16",
                          "sample": f"first {g_s} groups x {sreps} reps, groups block-sharded "
                                    f"over {th} threads"}
    return out


# ============================ single-kernel configurations ===================================
def _timed(eng, steps, warmup, launch, before=None):
    """warmup + steps launches on the engine stream; HIP events (engine runtime) around each
    launch on the stream the kernels run on; wall clock around the timed loop.
    Returns (wall_s, [ms per launch])."""
    for _ in range(warmup):
        if before:
            before()
        launch()
    eng.synchronize()
    evs = [(eng.event_create(), eng.event_create()) for _ in range(steps)]
    t0 = time.perf_counter()
    for e0, e1 in evs:
        if before:
            before()
        eng.event_record(e0)
        launch()
        eng.event_record(e1)
    eng.synchronize()
    wall = time.perf_counter() - t0
    ms = [eng.event_elapsed_ms(e0, e1) for e0, e1 in evs]
    for e0, e1 in evs:
        eng.event_destroy(e0)
        eng.event_destroy(e1)
    return wall, ms


def _cpu_loop(fn, budget=10.0, max_reps=20):
    secs, reps = 0.0, 0
    while secs < budget and reps < max_reps:
        secs += fn()
        reps += 1
    return secs, reps


def kernel_bench(a, rk):
    """BASELINE.json configs 2-4 and the §8(f) rows on one GPU (replicas only: under torchrun
    every rank runs its own copy of the workload and `value` sums the ranks)."""
    world, rank = rk.world, rk.rank
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as OL  # CPU oracle: the checker and the CPU baseline, never the measured path
    N = 5
    mode = R.MODE_MIN if a.mode == "min" else R.MODE_CLASSIC
    eng = Engine(rk.local, n_replicas=N, mode=mode, kv_capacity=a.kv_capacity or a.apply_keys,
                 apply_path={"auto": R.APPLY_AUTO, "small": R.APPLY_SMALL, "sorted": R.APPLY_SORTED,
                             "partitioned": R.APPLY_PARTITIONED}[a.apply_path])
    ar = Arena(eng)
    put, get, sync = ar.put, ar.get, eng.synchronize
    lib = OL.load()

    t_gen = time.time()
    host_call = None
    if a.workload == "tally":
        I = a.instances
        recs, st = synth.accept_replies(I, N, 0.7, seed=42)
        n = len(recs)
        d_recs, d_st = put(recs), put(st)
        d_out = ar.empty(len(st), R.INST_STATE)
        d_scal = ar.empty(1 + N, np.int32)
        scal0 = put(np.array([-1] + [0] * N, np.int32))
        d_dec = ar.empty(I, np.uint8)
        t_gen = time.time() - t_gen
        wall, ms = _timed(eng, a.steps, a.warmup,
                          lambda: eng.accept_tally_dev(d_recs.ptr, n, d_st.ptr, d_out.ptr, I, 0,
                                                       d_scal.ptr, d_dec.ptr, eng.stream),
                          before=lambda: eng.memcpy(d_scal.ptr, scal0.ptr, d_scal.nbytes, D2D))
        alg = n * 16 + I * 16 * 2  # replies + state in/out (96 B/instance)
        units, unit = I, "instances/s"
        kernel = f"k_accept_tile<{a.mode}>"
        kernel_pat = ["k_accept_tile"]
        o = OL.Oracle(N, mode)
        w_st, w_cu, w_pc, w_dec = o.accept_tally(recs, st, 0, -1)
        got_st = get(d_out)
        sc = get(d_scal)
        bit_exact = bool(np.array_equal(got_st.view(np.int32), w_st.view(np.int32))
                         and sc[0] == w_cu and np.array_equal(sc[1:], w_pc)
                         and np.array_equal(get(d_dec), w_dec))
        parity = {"instances_checked": I, "bit_exact": bit_exact}

        def cpu_once():
            s2 = st.copy()
            cu = C.c_int32(-1)
            pc = np.zeros(N, np.int32)
            return lib.orc_bench_accept(N, mode, recs.ctypes.data, n, s2.ctypes.data, I, 0,
                                        C.byref(cu), pc.ctypes.data) * 1e-9
        secs, reps = _cpu_loop(cpu_once)
        cpu = {"value": I * reps / secs, "unit": unit, "cores": 1, "kind": "port",
               "sample": f"the full workload ({I} instances, {n} replies) x {reps}, "
                         f"pointer-per-instance log, one thread, {secs:.1f} s timed"}
        workload = f"config2: {I} instances x {N - 1} AcceptReplies, N={N}, p_ok=0.7, mode {a.mode}"
    elif a.workload == "prepare":
        I = a.instances
        recs, st = synth.prepare_replies(I, N, 0.8, seed=43)
        n = len(recs)
        d_recs, d_st = put(recs), put(st)
        d_out = ar.empty(len(st), R.PREP_STATE)
        d_db = ar.empty(1, np.int32)
        db0 = put(np.array([-1], np.int32))
        d_prep = ar.empty(I, np.uint8)
        t_gen = time.time() - t_gen
        wall, ms = _timed(eng, a.steps, a.warmup,
                          lambda: eng.prepare_select_dev(d_recs.ptr, n, d_st.ptr, d_out.ptr, I, 0,
                                                         d_db.ptr, d_prep.ptr, eng.stream),
                          before=lambda: eng.memcpy(d_db.ptr, db0.ptr, 4, D2D))
        alg = n * 16 + I * 32 * 2  # 128 B/instance
        units, unit = I, "instances/s"
        kernel = "k_prepare_tile"
        kernel_pat = ["k_prepare_tile"]
        o = OL.Oracle(N, R.MODE_CLASSIC)
        t0 = time.perf_counter()
        w_st, w_db, w_prep = o.prepare_select(recs, st, 0, -1)
        t_orc = time.perf_counter() - t0
        bit_exact = bool(np.array_equal(get(d_out).view(np.int32), w_st.view(np.int32))
                         and int(get(d_db)[0]) == w_db and np.array_equal(get(d_prep), w_prep))
        parity = {"instances_checked": I, "bit_exact": bit_exact}

        def cpu_once():
            t0 = time.perf_counter()
            o.prepare_select(recs, st, 0, -1)
            return time.perf_counter() - t0
        secs, reps = _cpu_loop(cpu_once, 10.0 - t_orc)
        secs, reps = secs + t_orc, reps + 1
        cpu = {"value": I * reps / secs, "unit": unit, "cores": 1, "kind": "port",
               "sample": f"the full workload ({I} instances, {n} replies) x {reps} through the "
                         f"oracle's sequential handler loop (incl. its numpy copy-in/out), "
                         f"one thread, {secs:.1f} s timed"}
        workload = f"config3: {I} instances x {N - 1} PrepareReplies, N={N}, p_ok=0.8, random ballots"
    elif a.workload == "prepare_min":
        Gp = a.prep_groups
        recs, off, gst = synth.prepare_replies_min(Gp, N, seed=46)
        n = len(recs)
        pc = np.zeros(Gp * N, np.int32)
        d_recs, d_off, d_gst0, d_pc0 = put(recs), put(off), put(gst), put(pc)
        d_gst = ar.empty(Gp, R.GROUP_PREP_STATE)
        d_pc = ar.empty(Gp * N, np.int32)
        d_eff = ar.empty(n, R.PREPARE_EFFECT)
        t_gen = time.time() - t_gen

        def reset():  # the bookkeeping is updated in place: every launch starts from the input
            eng.memcpy(d_gst.ptr, d_gst0.ptr, d_gst.nbytes, D2D)
            eng.memcpy(d_pc.ptr, d_pc0.ptr, d_pc.nbytes, D2D)
        wall, ms = _timed(eng, a.steps, a.warmup,
                          lambda: eng.prepare_select_min_dev(d_recs.ptr, n, d_off.ptr, d_gst.ptr,
                                                             Gp, d_pc.ptr, d_eff.ptr, eng.stream),
                          before=reset)
        # replies + offsets in, group state in/out, peerCommits in/out, one effect per reply
        alg = n * 24 + (Gp + 1) * 8 + Gp * 32 * 2 + Gp * N * 4 * 2 + n * 8
        units, unit = Gp, "groups/s"
        kernel = "k_prepare_min"
        kernel_pat = ["k_prepare_min"]
        o = OL.Oracle(N, R.MODE_MIN)
        w_gst, w_pc, w_eff = o.prepare_select_min(recs, off, gst, pc)
        bit_exact = bool(np.array_equal(get(d_gst).view(np.int32), w_gst.view(np.int32))
                         and np.array_equal(get(d_pc), w_pc)
                         and np.array_equal(get(d_eff).view(np.int32), w_eff.view(np.int32)))
        parity = {"groups_checked": Gp, "bit_exact": bit_exact}

        def cpu_once():
            t0 = time.perf_counter()
            o.prepare_select_min(recs, off, gst, pc)
            return time.perf_counter() - t0
        secs, reps = _cpu_loop(cpu_once, 10.0, 200)
        cpu = {"value": Gp * reps / secs, "unit": unit, "cores": 1, "kind": "port",
               "sample": f"the full workload ({Gp} groups, {n} replies) x {reps} through the "
                         f"oracle's handlePrepareReply loop (incl. numpy copy-in/out), one "
                         f"thread, {secs:.1f} s timed"}
        workload = (f"config3 (MIN): {Gp} groups x {N - 1} PrepareReplies, one PrepareBookkeeping "
                    f"per group (latency-bound: reported, not roofline-graded)")
    elif a.workload == "apply":
        M, K = a.commands, a.apply_keys
        op, key, val = synth.commands(M, K, 0.5, a.dist, seed=44)
        d_op, d_key, d_val = put(op), put(key), put(val)
        d_ret = ar.empty(M, np.int64)
        d_conf = ar.empty(M, np.uint8)
        t_gen = time.time() - t_gen
        launch = lambda: eng.apply_dev(d_op.ptr, d_key.ptr, d_val.ptr, M, d_ret.ptr,  # noqa: E731
                                       d_conf.ptr, eng.stream)
        eng.apply_reserve(M)
        launch()  # the table holds every key from here on: every timed call does the same work
        sync()
        wall, ms = _timed(eng, a.steps, a.warmup, launch)
        n_keys = eng.kv_size()
        alg = M * (17 + 9) + n_keys * 16 * 2  # commands in, ret+conf out, table read + written
        units, unit = M, "commands/s"
        kernel = "mpx_apply pipeline"
        kernel_pat = ["mpx::", "rocprim"]
        if M <= R.APPLY_SMALL_MAX and a.apply_path in ("auto", "small"):
            # the device-pointer call is one kernel (the host forms' three, timed below for
            # host_call, are not part of the measured call)
            kernel, kernel_pat = "k_small_part", ["k_small_part"]
        o = OL.Oracle(N, mode)
        o.apply(op, key, val)
        w_ret, w_conf = o.apply(op, key, val)
        wk, wv = o.kv_export()
        order = np.argsort(wk, kind="stable")
        gk, gv = eng.kv_export()
        bit_exact = bool(np.array_equal(get(d_ret), w_ret) and np.array_equal(get(d_conf), w_conf)
                         and np.array_equal(gk, wk[order]) and np.array_equal(gv, wv[order]))
        parity = {"commands_checked": M, "bit_exact": bit_exact}
        if M <= 1 << 16:
            # a replica-sized call (one drained executeCommands batch, MAX_BATCH = 5000,
            # bareminpaxos.go:22): the synchronous host-pointer form the cgo shim calls, per
            # call (H2D of the commands, the launch(es), D2H of ret / conf), same table
            hc = []
            for _ in range(max(20, 4 * a.steps)):
                t0 = time.perf_counter()
                hr, hcf = eng.apply(op, key, val)
                hc.append(time.perf_counter() - t0)
            parity["host_form_bit_exact"] = bool(np.array_equal(hr, w_ret)
                                                 and np.array_equal(hcf, w_conf))
            host_call = {"median_us": float(np.median(hc)) * 1e6,
                         "min_us": float(np.min(hc)) * 1e6, "calls": len(hc),
                         "form": "mpx_apply (host pointers, synchronous)"}
            if M <= R.APPLY_SMALL_MAX and a.apply_path in ("auto", "small"):
                # the zero-copy form (mpx_apply_buffers / mpx_apply_staged): the shim builds the
                # drained batch straight in the engine's pinned arrays, so only the call is timed
                io = eng.apply_buffers(M)
                io["op"][:M], io["key"][:M], io["val"][:M] = op, key, val
                hs = []
                for _ in range(max(20, 4 * a.steps)):
                    t0 = time.perf_counter()
                    eng.apply_staged(M)
                    hs.append(time.perf_counter() - t0)
                parity["staged_form_bit_exact"] = bool(np.array_equal(io["ret"][:M], w_ret)
                                                       and np.array_equal(io["conf"][:M], w_conf))
                host_call["staged"] = {"median_us": float(np.median(hs)) * 1e6,
                                       "min_us": float(np.min(hs)) * 1e6, "calls": len(hs),
                                       "form": "mpx_apply_staged (engine-pinned arrays, "
                                               "synchronous)"}
        ret = np.zeros(M, np.int64)
        k0, v0 = np.ascontiguousarray(wk), np.ascontiguousarray(wv)
        secs, reps = _cpu_loop(lambda: lib.orc_bench_apply(
            k0.ctypes.data, v0.ctypes.data, len(k0), op.ctypes.data, key.ctypes.data,
            val.ctypes.data, M, ret.ctypes.data) * 1e-9)
        cpu = {"value": M * reps / secs, "unit": unit, "cores": 1, "kind": "port",
               "sample": f"the full workload ({M} commands over {K} keys, {a.dist}) x {reps}, "
                         f"Execute per command on an unordered_map, one thread, {secs:.1f} s timed"}
        workload = f"config4: {M} PUT/GET (p_put=0.5) over {K} keys, {a.dist}"
        if M <= 1 << 16:
            workload = (f"apply (replica batch): {M} PUT/GET (p_put=0.5) over {K} keys, "
                        f"{a.dist}, path {a.apply_path}")
    elif a.workload == "conflict":
        M, K, Bc = a.commands, a.apply_keys, 4
        op, key, _ = synth.commands(M, K, 0.5, a.dist, seed=44)
        n_inst = M // Bc
        off = (np.arange(n_inst + 1, dtype=np.uint64) * np.uint64(Bc))
        d_op, d_key, d_off = put(op), put(key), put(off)
        d_out = ar.empty(max(n_inst - 1, 1), np.uint8)
        t_gen = time.time() - t_gen
        wall, ms = _timed(eng, a.steps, a.warmup,
                          lambda: eng.conflict_batch_dev(d_op.ptr, d_key.ptr, d_off.ptr, n_inst,
                                                         d_out.ptr, eng.stream))
        # every command is read by the pairs it belongs to (twice), offsets once, one flag out
        alg = M * 9 + (n_inst + 1) * 8 + (n_inst - 1)
        units, unit = n_inst - 1, "instance pairs/s"
        kernel = "k_conflict_batch"
        kernel_pat = ["k_conflict_batch"]
        o = OL.Oracle(N, mode)
        want = o.conflict_batch(op, key, off)
        bit_exact = bool(np.array_equal(get(d_out, n_inst - 1), want))
        parity = {"pairs_checked": n_inst - 1, "bit_exact": bit_exact}
        cout = np.zeros(max(n_inst - 1, 1), np.uint8)

        def cpu_once():
            t0 = time.perf_counter()
            lib.orc_conflict_batch(op.ctypes.data, key.ctypes.data, off.ctypes.data, n_inst,
                                   cout.ctypes.data)
            return time.perf_counter() - t0
        secs, reps = _cpu_loop(cpu_once)
        cpu = {"value": (n_inst - 1) * reps / secs, "unit": unit, "cores": 1, "kind": "port",
               "sample": f"the full run ({n_inst} instances of {Bc} commands) x {reps}, the "
                         f"nested ConflictBatch loop per pair, one thread, {secs:.1f} s timed"}
        workload = (f"conflict: ConflictBatch(inst i, inst i+1) over {n_inst} instances of {Bc} "
                    f"config-4 commands ({a.dist} keys over {K})")
    elif a.workload == "fanout":
        M, Cn = a.commands, a.clients
        recs = synth.replies(M, Cn, seed=55)
        d_recs = put(recs)
        d_out = ar.empty(M * R.PROPOSE_REPLY_BYTES, np.uint8)
        d_off = ar.empty(Cn + 1, np.uint64)
        eng.encode_replies_reserve(M)
        t_gen = time.time() - t_gen
        wall, ms = _timed(eng, a.steps, a.warmup,
                          lambda: eng.encode_replies_dev(d_recs.ptr, M, Cn, 1, 0, d_out.ptr,
                                                         d_off.ptr, eng.stream))
        alg = M * (24 + R.PROPOSE_REPLY_BYTES) + (Cn + 1) * 8  # records in, wire bytes out
        units, unit = M, "replies/s"
        kernel = "mpx_encode_replies pipeline"
        kernel_pat = ["mpx::", "rocprim"]
        o = OL.Oracle(N, mode)
        w_out, w_off = o.encode_replies(recs, Cn, 1, 0)
        bit_exact = bool(get(d_out).tobytes() == w_out.tobytes()
                         and np.array_equal(get(d_off), w_off))
        parity = {"replies_checked": M, "bit_exact": bit_exact}
        cout = np.zeros(M * R.PROPOSE_REPLY_BYTES, np.uint8)
        coff = np.zeros(Cn + 1, np.uint64)

        def cpu_once():
            t0 = time.perf_counter()
            lib.orc_encode_replies(recs.ctypes.data, M, Cn, 1, 0, cout.ctypes.data,
                                   coff.ctypes.data)
            return time.perf_counter() - t0
        secs, reps = _cpu_loop(cpu_once)
        cpu = {"value": M * reps / secs, "unit": unit, "cores": 1, "kind": "port",
               "sample": f"the full batch ({M} replies over {Cn} connections) x {reps}, one "
                         f"Marshal per reply into per-connection buffers, one thread, "
                         f"{secs:.1f} s timed"}
        workload = f"fanout: {M} ProposeReplyTS over {Cn} client connections"
    elif a.workload == "log":
        I = a.instances
        fmt = R.LOG_CATCHUP if a.log_format == "catchup" else R.LOG_DURABLE
        recs, coff, op, key, val = synth.log_records(I, 4, seed=58)
        M = len(op)
        d_recs, d_off, d_op, d_key, d_val = put(recs), put(coff), put(op), put(key), put(val)
        bound = eng.lib.mpx_encode_log_bound(I, M)
        d_out = ar.empty(bound, np.uint8)
        d_ro = ar.empty(I + 1, np.uint64)
        eng.encode_log_reserve(I, M)
        t_gen = time.time() - t_gen
        wall, ms = _timed(eng, a.steps, a.warmup,
                          lambda: eng.encode_log_dev(fmt, d_recs.ptr, I, d_off.ptr, d_op.ptr,
                                                     d_key.ptr, d_val.ptr, M, d_out.ptr, d_ro.ptr,
                                                     eng.stream))
        o = OL.Oracle(N, mode)
        w_out, w_ro = o.encode_log(fmt, recs, coff, op, key, val)
        total = int(w_ro[-1])
        # records + offsets + commands in, the encoding + record offsets out
        alg = I * (16 + 8) + M * 17 + total + (I + 1) * 8
        units, unit = I, "instances/s"
        kernel = "mpx_encode_log pipeline"
        kernel_pat = ["mpx::", "rocprim"]
        bit_exact = bool(np.array_equal(get(d_ro), w_ro)
                         and get(d_out, total).tobytes() == w_out.tobytes())
        parity = {"instances_checked": I, "bytes": total, "bit_exact": bit_exact}
        cout = np.zeros(total, np.uint8)
        cro = np.zeros(I + 1, np.uint64)

        def cpu_once():
            t0 = time.perf_counter()
            lib.orc_encode_log(fmt, recs.ctypes.data, I, coff.ctypes.data, op.ctypes.data,
                               key.ctypes.data, val.ctypes.data, cout.ctypes.data, total,
                               cro.ctypes.data)
            return time.perf_counter() - t0
        secs, reps = _cpu_loop(cpu_once)
        cpu = {"value": I * reps / secs, "unit": unit, "cores": 1, "kind": "port",
               "sample": f"the full run ({I} instances, {M} commands, {total} bytes) x {reps}, "
                         f"one Marshal per instance and command, one thread, {secs:.1f} s timed"}
        workload = f"log ({a.log_format}): {I} committed instances x 4 commands, {total} bytes"
    elif a.workload == "replay":
        I = a.instances
        recs, coff, op, key, val = synth.log_records(I, 1, seed=59)
        recs = recs.copy()
        rng = np.random.default_rng(60)
        recs["inst_no"] = (rng.integers(0, I // 2, I) if a.replay_dups else rng.permutation(I)
                           ).astype(np.int32)
        o = OL.Oracle(N, mode)
        log, _ = o.encode_log(R.LOG_DURABLE, recs, coff, op, key, val)
        L = len(log)
        d_log = put(log)
        d_recs = ar.empty(I, R.LOG_REC)
        d_op = ar.empty(I, np.uint8)
        d_key = ar.empty(I, np.int64)
        d_val = ar.empty(I, np.int64)
        d_last = ar.full(I, np.int32, 0xFF)
        d_sc = put(np.array([0, -1], np.int32))
        if not a.replay_atomic:
            eng.replay_durable_reserve(L, I)  # the binned slot maximum's scratch
        t_gen = time.time() - t_gen
        # every output is idempotent under repetition (slots and watermarks are maxima)
        wall, ms = _timed(eng, a.steps, a.warmup,
                          lambda: eng.replay_durable_dev(d_log.ptr, L, I, d_recs.ptr, d_op.ptr,
                                                         d_key.ptr, d_val.ptr, d_last.ptr,
                                                         d_sc.ptr, eng.stream))
        w = o.replay_durable(log, I)
        # log read once; records, op, key, val written once; one 4-byte slot per record
        alg = L + I * (16 + 1 + 8 + 8) + I * 4
        units, unit = I, "records/s"
        kernel = "k_replay_durable"
        kernel_pat = ["k_replay_durable", "k_rb_", "k_scan_"]
        bit_exact = bool(np.array_equal(get(d_recs), w[0]) and np.array_equal(get(d_op), w[1])
                         and np.array_equal(get(d_key), w[2]) and np.array_equal(get(d_val), w[3])
                         and np.array_equal(get(d_last), w[4])
                         and get(d_sc).tolist() == [w[5], w[6]])
        parity = {"records_checked": I, "bytes": L, "bit_exact": bit_exact}
        c = [np.zeros(I, R.LOG_REC), np.zeros(I, np.uint8), np.zeros(I, np.int64),
             np.zeros(I, np.int64), np.zeros(I, np.int32), np.zeros(2, np.int32)]

        def cpu_once():
            c[4][:] = -1
            c[5][:] = (0, -1)
            t0 = time.perf_counter()
            lib.orc_replay_durable(log.ctypes.data, L, I, 0, *[x.ctypes.data for x in c])
            return time.perf_counter() - t0
        secs, reps = _cpu_loop(cpu_once)
        cpu = {"value": I * reps / secs, "unit": unit, "cores": 1, "kind": "port",
               "sample": f"the full log ({I} records, {L} bytes) x {reps} through the oracle's "
                         f"getDataFromStableStore loop, one thread, {secs:.1f} s timed"}
        workload = (f"replay (durable): {I} records x 1 command, {L} bytes, instNo "
                    + ("drawn with repeats over I/2 slots" if a.replay_dups else "a permutation"))
    elif a.workload == "stream":
        from minpaxos_amd import wire
        I = a.instances
        recs, _ = synth.accept_replies(I, N, 0.7, seed=42)
        buf = wire.leader_stream(mode, recs, seed=61, prepare_every=a.prepare_every,
                                 n_cmds=a.prep_cmds)
        L = len(buf)
        o = OL.Oracle(N, mode)
        w = o.decode_stream(buf)
        n_ar, n_pr, n_var, n_oth = (len(x) for x in w[:4])
        d_buf = put(buf)
        d_ar = ar.empty(max(n_ar, 1), R.ACCEPT_REPLY)
        pdt = R.PREPARE_REPLY_MIN if mode == R.MODE_MIN else R.PREPARE_REPLY
        d_pr = ar.empty(max(n_pr, 1), pdt)
        d_var = ar.empty(max(n_var, 1), R.VAR_FRAME)
        d_oth = ar.empty(max(n_oth, 1), R.PEER_FRAME)
        d_res = ar.full(1, R.STREAM_RESULT, 0)
        out = _lib.MpxDecodeOut(d_ar.ptr, n_ar, d_pr.ptr, n_pr, d_var.ptr, n_var, d_oth.ptr, n_oth)
        eng.decode_stream_reserve(L)
        t_gen = time.time() - t_gen
        wall, ms = _timed(eng, a.steps, a.warmup,
                          lambda: eng.decode_stream_dev(d_buf.ptr, L, 0, out, d_res.ptr,
                                                        eng.stream),
                          before=lambda: eng.memset(d_res.ptr, 0, d_res.nbytes))
        # stream read once, records written once
        alg = L + n_ar * 16 + n_pr * pdt.itemsize + n_var * 32 + n_oth * 8
        units, unit = n_ar + n_pr, "replies/s"
        kernel = "mpx_decode_stream pipeline"
        kernel_pat = ["mpx::"]
        got = [get(d_ar, n_ar), get(d_pr, n_pr), get(d_var, n_var), get(d_oth, n_oth), get(d_res)[0]]
        bit_exact = all(g.tobytes() == x.tobytes() for g, x in zip(got[:4], w[:4])) and all(
            int(got[4][f]) == int(w[4][f]) for f in ("consumed", "n_accept_replies",
                                                     "n_prepare_replies", "n_var", "n_other",
                                                     "stop_reason", "stop_code"))
        parity = {"frames_checked": n_ar + n_var + n_oth, "bytes": L, "bit_exact": bool(bit_exact)}
        car = np.zeros(max(n_ar, 1), R.ACCEPT_REPLY)
        cpr = np.zeros(max(n_pr, 1), pdt)
        cvar = np.zeros(max(n_var, 1), R.VAR_FRAME)
        coth = np.zeros(max(n_oth, 1), R.PEER_FRAME)
        cres = np.zeros(1, R.STREAM_RESULT)
        cout = _lib.MpxDecodeOut(car.ctypes.data, n_ar, cpr.ctypes.data, n_pr, cvar.ctypes.data,
                                 n_var, coth.ctypes.data, n_oth)

        def cpu_once():
            t0 = time.perf_counter()
            lib.orc_decode_stream(mode, buf.ctypes.data, L, C.byref(cout), cres.ctypes.data)
            return time.perf_counter() - t0
        secs, reps = _cpu_loop(cpu_once)
        cpu = {"value": (n_ar + n_pr) * reps / secs, "unit": unit, "cores": 1, "kind": "port",
               "sample": f"the full stream ({L} bytes) x {reps} through the oracle's "
                         f"replicaListener + Unmarshal loop, one thread, {secs:.1f} s timed"}
        workload = (f"stream ({a.mode} wire): {n_ar} AcceptReplies + {n_pr} PrepareReplies "
                    f"({a.prep_cmds} Commands each, one per {a.prepare_every} AcceptReplies) + "
                    f"{n_oth} Beacons, {L} bytes")
    else:  # decode
        I = a.instances
        recs, _ = synth.accept_replies(I, N, 0.7, seed=42)
        buf = synth.peer_stream(recs, seed=52, p_beacon=1.0 / 4096)
        L = len(buf)
        o = OL.Oracle(N, mode)
        w_ar, w_oth, w_res = o.decode_peer_stream(buf)
        n_ar, n_oth = int(w_res["n_accept_replies"]), int(w_res["n_other"])
        d_buf = put(buf)
        d_ar = ar.empty(n_ar, R.ACCEPT_REPLY)
        d_oth = ar.empty(max(n_oth, 1), R.PEER_FRAME)
        d_res = ar.empty(1, R.DECODE_RESULT)
        eng.decode_reserve(L)
        t_gen = time.time() - t_gen
        wall, ms = _timed(eng, a.steps, a.warmup,
                          lambda: eng.decode_peer_stream_dev(d_buf.ptr, L, d_ar.ptr, n_ar,
                                                             d_oth.ptr, n_oth, d_res.ptr,
                                                             eng.stream))
        alg = L + n_ar * 16 + n_oth * 8  # stream read once, records written once
        units, unit = n_ar, "AcceptReplies/s"
        kernel = "mpx_decode_peer_stream pipeline"
        kernel_pat = ["mpx::"]
        bit_exact = bool(get(d_res).tobytes() == w_res.tobytes()
                         and get(d_ar).tobytes() == w_ar.tobytes()
                         and get(d_oth, n_oth).tobytes() == w_oth.tobytes())
        parity = {"frames_checked": n_ar + n_oth, "bytes": L, "bit_exact": bit_exact}
        car = np.zeros(n_ar, R.ACCEPT_REPLY)
        coth = np.zeros(max(n_oth, 1), R.PEER_FRAME)
        cres = np.zeros(1, R.DECODE_RESULT)

        def cpu_once():
            t0 = time.perf_counter()
            lib.orc_decode_peer_stream(buf.ctypes.data, L, car.ctypes.data, n_ar,
                                       coth.ctypes.data, n_oth, cres.ctypes.data)
            return time.perf_counter() - t0
        secs, reps = _cpu_loop(cpu_once)
        cpu = {"value": n_ar * reps / secs, "unit": unit, "cores": 1, "kind": "port",
               "sample": f"the full stream ({L} bytes, {n_ar} AcceptReplies, {n_oth} Beacons) "
                         f"x {reps} through the oracle's replicaListener loop, one thread, "
                         f"{secs:.1f} s timed"}
        workload = (f"decode: {n_ar} AcceptReply frames (config-2 replies, {I} instances) + "
                    f"{n_oth} Beacons, {L} bytes")
    wall = rk.max(wall)
    kern_avg = float(np.mean(ms))
    kern_med = float(np.median(ms))
    achieved = alg / (kern_avg * 1e-3) / 1e9
    # the exact configuration a counter pass must have been taken on
    tkey = {"workload": a.workload, "mode": a.mode}
    tkey.update({
        "tally": lambda: {"instances": a.instances, "replicas": N},
        "prepare": lambda: {"instances": a.instances},
        "prepare_min": lambda: {"groups": a.prep_groups},
        "apply": lambda: {"commands": a.commands, "apply_keys": a.apply_keys, "dist": a.dist,
                          "kv_capacity": a.kv_capacity or a.apply_keys, "apply_path": a.apply_path},
        "conflict": lambda: {"commands": a.commands, "apply_keys": a.apply_keys, "dist": a.dist},
        "decode": lambda: {"instances": a.instances},
        "stream": lambda: {"instances": a.instances, "prepare_every": a.prepare_every,
                           "prep_cmds": a.prep_cmds},
        "fanout": lambda: {"commands": a.commands, "clients": a.clients},
        "log": lambda: {"instances": a.instances, "log_format": a.log_format},
        "replay": lambda: {"instances": a.instances, "replay_dups": bool(a.replay_dups),
                           **({"replay_atomic": True} if a.replay_atomic else {})},
    }[a.workload]())
    traffic, tnote = traffic_for(tkey, alg, a.traffic_json)
    rl = {"bound": "hbm", "kernel": kernel, "achieved": achieved,
          "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": achieved / PEAK_HBM_GBS,
          "traffic": traffic, "traffic_note": tnote, "traffic_key": tkey,
          "traffic_kernels": kernel_pat, "alg_bytes_per_launch": alg,
          "kernel_ms_avg": kern_avg, "kernel_ms_median": kern_med,
          "kernel_ms_min": float(np.min(ms)),
          "frac_at_median": alg / (kern_med * 1e-3) / 1e9 / PEAK_HBM_GBS}
    if a.workload in ISSUE_BOUND:
        # the framing DP (decode, stream) and the fan-out's per-reply LDS ranking are bound by
        # instruction issue, not HBM: graded against the issue peaks
        rl = dict(issue_roofline(kernel, tkey, kern_avg, {k: rl[k] for k in (
            "achieved", "peak", "unit", "frac", "traffic", "traffic_note")}, a.traffic_json),
                  traffic_key=tkey, traffic_kernels=kernel_pat, alg_bytes_per_launch=alg,
                  kernel_ms_avg=kern_avg, kernel_ms_median=kern_med,
                  kernel_ms_min=float(np.min(ms)))
    if rank == 0:
        line = {
            "metric": f"{a.workload} throughput ({unit})", "value": units * a.steps * world / wall,
            "unit": unit, "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": wall / a.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "int32/int64", "data": "synthetic (splitmix64)",
            "config": {"workload": workload, "parallelism": f"replicas x{world}"},
            "roofline": rl,
            "gen_s": round(t_gen, 2), "parity": parity, "runtime": _lib.runtime_info(),
            **({"host_call": host_call} if host_call else {}),
            # calls of the measured pipeline this process made (the counter collector divides
            # by it): warm-up + timed, plus apply's table-filling first call
            "launches_in_process": a.warmup + a.steps + (1 if a.workload == "apply" else 0),
        }
        if world == 1 and not a.no_cpu_baseline:
            line["cpu_baseline"] = cpu
        print(json.dumps(line), flush=True)
    ar.close()
    eng.close()


if __name__ == "__main__":
    main()
