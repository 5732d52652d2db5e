#!/usr/bin/env python3
"""Benchmark of the MI355X path tracer on BASELINE.json's headline config.

Metric: Mrays/s at 1920x1080, 8 bounces (C2: Cornell box, 5 quads + 2 spheres, 64 spp per frame),
with the per-pixel RMSE vs the CPU oracle (reference semantics) reported beside it.

One step = one 64-spp C2 frame rendered by the HIP megakernel, one process per GPU.

* N = 1: the whole frame on one GPU.
* N > 1, --scaling strong (default; C3 of BASELINE.json): the pixel rows of ONE frame
  are dealt cyclically over the ranks (row y -> rank y mod N; RNG streams are keyed by the global
  pixel id, path_tracer.cu:36-46/336-339, so the assembled frame is bit-identical to the 1-GPU frame)
  and every step ends with an RCCL gather over xGMI of the presented BGRA8 framebuffer to rank 0
  (--gather frame; the reference reads this buffer back every frame, path_tracer.cu:385) or of the
  float accumulators (--gather accum). After the timed steps the float accumulators are gathered
  once and checked.
* N > 1, --scaling weak (opt-in): every rank renders the full frame with its own RNG streams (seed
  1984 + rank): N independent estimates, no collective in the timed region.

value = closest-hit queries traced by all ranks in the K timed steps / the max over ranks of the
barrier-bracketed wall time.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2] [--scaling strong|weak]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Without torch.distributed.run, --gpus N > 1 starts its N rank processes itself (before anything
touches the GPU) and returns rank 0's JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "path-tracer-and-rasterizer-engine_amd"))

FP32_PEAK_TFLOPS = 157.3        # MI355X FP32 vector peak (MI355X_MICROARCH.md); the path runs on the VALU
HBM_PEAK_GBPS = 8000.0          # MI355X HBM3E peak, MI355X_MICROARCH.md
STREAMED_CONFIGS = ("c4", "c5")  # scenes past the LDS: the first kTuneLaunches (4) launches time both camera-ray paths


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100,
                    help="timed steps (default 100: the timed region starts and ends with an idle GPU, and the "
                         "overlapped launches' fill and drain — about one launch less one step — is spread over K "
                         "steps: C2 0.884 ms per step at K = 20, 0.848-0.859 at K = 40, tools/RUNS.md r06 run 42)")
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed steps (default 10; 5 for the streamed configs c4 / c5, whose first 4 launches time "
                         "both camera-ray paths, DESIGN.md §3.5)")
    ap.add_argument("--config", default="c2")
    ap.add_argument("--spp", type=int, default=0,
                    help="samples per pixel per step (default: the config's; a progressive pass of C5's 1024)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=60.0,
                    help="wall time of the CPU-baseline sample (a bounded sample: the default run stays within "
                         "minutes; BASELINE.md §3's 60-s runs: --cpu-seconds 60)")
    ap.add_argument("--verify-rows", type=int, default=16)
    ap.add_argument("--pmc-json", default="",
                    help="PMC traffic of the config's launch (tools/pmc_traffic.py; default: the newest "
                         "profiles/r0*/pmc_traffic_<config>*.json whose spp_per_launch equals this run's)")
    ap.add_argument("--pmc-mix-json", default="",
                    help="rocprofv3 instruction-mix counters of the same kernel (VALU pipe occupancy; default: the "
                         "newest profiles/r0*/<config>_pmc_mix*.json)")
    ap.add_argument("--work-json", default="",
                    help="executed-work counters of the config (tools/work_counters.py; default "
                         "profiles/r02/work_<config>.json): prices C4/C5, reported beside C2's algorithmic price")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend for N > 1 (nccl = RCCL over xGMI; gloo = rehearsal)")
    ap.add_argument("--one-device", action="store_true",
                    help="all ranks on GPU 0 (multi-rank rehearsal on a 1-GPU box; use with --backend gloo)")
    ap.add_argument("--save-frame", default="", help="rank 0 writes the assembled float frame (.npy)")
    ap.add_argument("--scaling", default="strong", choices=["weak", "strong"],
                    help="strong (default): rows of one frame + gather; weak: every rank a full frame, seed 1984+rank")
    ap.add_argument("--gather", default="frame", choices=["frame", "accum"],
                    help="what the strong-scaling step gathers to rank 0: the BGRA8 frame or the float accumulators")
    ap.add_argument("--overlap", default="auto", choices=["auto", "off"],
                    help="overlapped launches on two streams (iqpt_set_overlap, DESIGN.md §3.8)")
    ap.add_argument("--certain", default="on", choices=["on", "off"],
                    help="A/B: certain pixels folded at once (iqpt_debug_set_certain, DESIGN.md §3.3)")
    ap.add_argument("--sky", default="on", choices=["on", "off"],
                    help="A/B: certain-miss pixels in iqpt_sky_kernel (iqpt_debug_set_sky, DESIGN.md §3.12)")
    ap.add_argument("--kernel-options", type=lambda v: int(v, 0), default=0,
                    help="A/B: render-kernel option mask (iqpt_debug_set_kernel_options; 0 = production)")
    ap.add_argument("--gather-sync", action="store_true",
                    help="N > 1: the blocking frame copy + gather of round 1 instead of the stream-ordered one")
    ap.add_argument("--lib", default="", help="A/B only: load this prebuilt libiqpt (compile-time knob builds)")
    ap.add_argument("--share-of", type=int, default=0,
                    help="rehearsal at N = 1: render rank 0's rows of an N-way C3 split (one GPU's share; "
                         "with --self-gather the per-step gather path too)")
    ap.add_argument("--gather-ctas", type=int, default=None,
                    help="A/B: RCCL blocks per frame gather (ncclConfig_t::maxCTAs; 0: RCCL's choice; "
                         "default: the library's)")
    ap.add_argument("--gather-prio", type=int, default=None, choices=[-1, 0, 1],
                    help="A/B: the communicator stream's priority (0: the library default)")
    ap.add_argument("--gather-skip", type=int, default=0, choices=range(8),
                    help="measurement only (wrong frames): 1 leaves out the collective, 2 the root's assembly, "
                         "4 the render streams' waits for the frame copies")
    ap.add_argument("--sky-order", choices=["ahead", "behind"], default=None,
                    help="A/B: overlapped launches run the sky kernel ahead of or behind the plain kernel "
                         "(default: the library's, behind)")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="A/B: no timing events around launches (kernel times and the roofline read 0)")
    ap.add_argument("--self-gather", action="store_true",
                    help="test: run the per-step gather path at N = 1 (a one-rank process group)")
    ap.add_argument("--two-ray", type=int, default=None, choices=[0, 1],
                    help="A/B: resident plain launches trace the path ray and the next sample's camera ray together "
                         "(iqpt_debug_set_two_ray; default: the library's, on)")
    ap.add_argument("--anyhit", type=int, default=None, choices=[0, 1],
                    help="A/B: any-hit queries for triangle-only scenes (iqpt_debug_set_anyhit; default: the library's, on)")
    ap.add_argument("--pixel-masks", type=int, default=None, choices=[0, 1, 2],
                    help="A/B: per-pixel candidate masks over streamed tile lists (iqpt_debug_set_pixel_masks: 0 none, "
                         "1 in the plain kernel, 2 the library's default: + iqpt_anyhit_kernel for any-hit scenes)")
    ap.add_argument("--stream-refill", type=int, default=None,
                    help="A/B: idle lanes before a streamed-scene wave takes new pixels (iqpt_debug_set_stream_refill; 1..64)")
    ap.add_argument("--stream-xcd", type=int, default=None, choices=[0, 1, 2, 3],
                    help="A/B: streamed scenes' tiles per XCD (iqpt_debug_set_stream_xcd: 0 one queue, 1 cost order "
                         "dealt to the XCDs, 2 bands of tile rows dealt to the XCDs, 3 the default: 1 up to 4 spp per launch)")
    ap.add_argument("--resident-refill", type=int, default=None,
                    help="A/B: idle lanes before a resident-scene wave takes new pixels (iqpt_debug_set_resident_refill)")
    ap.add_argument("--spec-margin", type=int, default=None,
                    help="A/B: spec windows' margin, 1 / this of the extra slots (iqpt_debug_set_spec; default 16)")
    ap.add_argument("--spec-parity", type=float, default=None,
                    help="A/B: spec parity pixels' threshold in slots per sample (iqpt_debug_set_spec_parity; 0 = every "
                         "slot traced, the round-4 kernel; default: the library's 1.875)")
    ap.add_argument("--split", default="auto", choices=["auto", "on", "off", "spec"],
                    help="sample-parallel chains (iqpt_set_split, DESIGN.md §3.7)")
    args = ap.parse_args()
    if args.warmup is None:
        args.warmup = 5 if args.config in STREAMED_CONFIGS else 10
    return args


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(args) -> int:
    """--gpus N > 1 without a launcher: start N fresh rank processes (nothing here has touched the GPU)
    with the torch.distributed environment, wait for all, return the worst exit code. A failing rank
    ends the others (their exact PIDs), so no rank waits forever in a collective."""
    port = _free_port()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve())] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0:
                rc = rc or code
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


def cpu_info() -> dict:
    model = ""
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"cpu_model": model, "cpus_visible": os.cpu_count()}


def baseline_threads() -> int:
    """The CPU share of this GPU: OMP_NUM_THREADS where the harness sets it (16 per GPU on the MI355X
    boxes), else every CPU this process may run on."""
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return env or len(os.sched_getaffinity(0))


def cpu_baseline(cfg, pk, cam, seconds: float) -> dict:
    """The oracle (the reference kernel restated as a host loop, OpenMP, same per-ray work) on the same
    scene: full-frame 1-spp passes until `seconds` of wall time (Mrays/s does not depend on spp)."""
    sys.path.insert(0, str(REPO / "oracle"))
    import oracle  # cpu_baseline leg only
    from iqpt import _build
    threads = baseline_threads()
    # -O3 -march=native, built here for this host's CPU; the parity build (no -march) if that fails
    try:
        _, build = _build.build_oracle_native()
        flavour = "native"
    except (RuntimeError, OSError) as e:
        build, flavour = f"the parity build liboracle.so (-march=native build failed: {str(e)[:120]})", "b"
    fr = oracle.OracleFrame(cfg.width, cfg.height, max_depth=cfg.max_depth, flavour=flavour)
    rays = 0
    passes = 0
    t0 = time.perf_counter()
    while True:
        rays += fr.render(pk, cam, 1, threads=threads)
        passes += 1
        dt = time.perf_counter() - t0
        if dt >= seconds:
            break
    info = cpu_info()
    return {"value": rays / dt / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
            "per_core": rays / dt / 1e6 / threads, **info, "build": build, "seconds": round(dt, 1),
            # the GPU box runs a command on its per-GPU CPU share (OMP_NUM_THREADS = 16 of the host's CPUs): the
            # host-wide figure is that share's rate scaled linearly to every visible CPU, stated, not measured
            "all_cpus_linear_estimate": round(rays / dt / 1e6 / threads * (info.get("cpus_visible") or threads), 1),
            "sample": f"{passes} full {cfg.width}x{cfg.height} 1-spp passes of {cfg.preset} "
                      f"(max_depth {cfg.max_depth}) in {dt:.1f} s, {rays} rays, {threads} OpenMP threads"}


def verify_vs_oracle(cfg, pk, cam, lin_rank, rank, world, nrows, seed=1984, spp=None) -> dict:
    """After the first frame: compare a band of this rank's rows with the oracle. `rank` and `world`
    describe the row partition (world 1 = the rank owns the whole frame)."""
    import iqpt
    sys.path.insert(0, str(REPO / "oracle"))
    import numpy as np
    import oracle
    y_band = int(cfg.height * 0.46)                     # through both spheres
    first = y_band + ((rank - y_band) % world)          # first row >= y_band owned by this rank
    k0 = (first - rank) // world
    ps = iqpt.pixel_set(cfg.width, cfg.height, 0, cfg.width, first, world, nrows)
    fr = oracle.OracleFrame(cfg.width, cfg.height, pixels=ps, seed=seed, max_depth=cfg.max_depth)
    fr.render(pk, cam, spp or cfg.spp)
    mine = lin_rank.reshape(-1, cfg.width, 4)[k0:k0 + nrows].reshape(-1, 4)
    a = mine[:, :3].astype(np.float64)
    b = fr.lin[:, :3].astype(np.float64)
    rmse = float(np.sqrt(np.mean((a - b) ** 2)))
    same = np.all(mine[:, :3].view(np.uint32) == fr.lin[:, :3].view(np.uint32), axis=1)
    return {"rmse": rmse, "bitexact_frac": float(same.mean()), "pixels": int(mine.shape[0])}


def load_json(path: str, cfg_name: str):
    p = Path(path) if path else None
    if not p or not p.exists():
        return None
    try:
        d = json.loads(p.read_text())
    except (OSError, ValueError):
        return None
    return d if d.get("config") == cfg_name else None


BYTES_PER_PIXEL_LAUNCH = 84     # RNG 24 read + 24 written, accumulator 16 + 16, BGRA8 4


def _by_sha(cands, accept):
    """The candidate profiles `accept` takes, the newest one of THESE kernel sources (kernel_sha16 equal to the
    build's) first, else the newest of any (reported as stale). Returns (profile, path, same_sources) or None."""
    from iqpt._build import kernel_source_sha16
    want = kernel_source_sha16()
    ok = [(d, c) for c in cands for d in [accept(c)] if d]
    for d, c in ok:
        if d.get("kernel_sha16") == want:
            return d, c, True
    return (ok[0][0], ok[0][1], False) if ok else None


def _rel(c: Path) -> str:
    c = c.resolve()
    return str(c.relative_to(REPO)) if c.is_relative_to(REPO) else str(c)


def find_pmc(cfg_name: str, spp: int, explicit: str):
    """The PMC traffic profile of THIS launch shape: same config and same samples per launch (traffic
    per launch grows with spp only through the kernel's own re-reads, but a 1-spp profile divided by a
    16-spp kernel time is meaningless), of these kernel sources where one exists. Returns (profile, path,
    same_sources) or (None, why, None)."""
    cands = [Path(explicit)] if explicit else sorted(
        (REPO / "profiles").glob(f"r0*/pmc_traffic_{cfg_name}*.json"), key=lambda q: (q.parent.name, q.name), reverse=True)
    why = ["no PMC profile of this config"]

    def accept(c):
        d = load_json(str(c), cfg_name)
        if d and d.get("spp_per_launch") != spp:
            why[0] = f"{_rel(c)} was taken at {d.get('spp_per_launch')} spp per launch, this run launches {spp}"
            return None
        return d
    got = _by_sha(cands, accept)
    return (got[0], _rel(got[1]), got[2]) if got else (None, why[0], None)


def find_mix(cfg_name: str, explicit: str):
    """The PMC instruction-mix profile (tools/pmc_mix.py) of this config's kernel: the explicit file, else the
    newest profiles/r0*/<config>_pmc_mix*.json of these kernel sources, else the newest of any. Returns
    (profile, path, same_sources)."""
    cands = [Path(explicit)] if explicit else sorted(
        (REPO / "profiles").glob(f"r0*/{cfg_name}_pmc_mix*.json"), key=lambda q: (q.parent.name, q.name), reverse=True)
    got = _by_sha(cands, lambda c: load_json(str(c), cfg_name))
    return (got[0], _rel(got[1]), got[2]) if got else (None, None, None)


def certain_pixels(pt, _lib) -> int:
    """Pixels of this context whose camera rays the certain-pixel proof resolves (0 when the path is off or
    the scene is streamed)."""
    import ctypes as C
    lb = _lib.load()
    lb.iqpt_debug_certain_tiles.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                            C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.c_uint32]
    n, nt, ntx = C.c_uint32(0), C.c_uint32(0), C.c_uint32(0)
    _lib.check(lb.iqpt_debug_certain_tiles(pt.handle, C.byref(n), C.byref(nt), C.byref(ntx), None, 0),
               "iqpt_debug_certain_tiles")
    return int(n.value)


# the kernels a launch mode runs (iqpt_debug_split_info's launch mode)
LAUNCH_KERNELS = {"plain": "iqpt_render_kernel", "anyhit": "iqpt_anyhit_kernel",
                  "spec": "iqpt_spec_kernel + iqpt_fan_kernel",
                  "split": "iqpt_render_kernel (split rounds)",
                  "split+fan": "iqpt_render_kernel (split rounds) + iqpt_fan_kernel"}


def mix_for_launch(cfg_name: str, launch_mode: str, split_ways: int, explicit: str):
    """The instruction-mix profile of the kernels this launch mode ran: the plain kernel's for a full-frame
    plain line; for a spec line the spec and fan kernels' own at this share (profiles/r0*/pmc_mix_{spec,fan}_n<N>.json,
    taken at the same C3 share); else none (no profile of those kernels). Returns (busy, split, source, same_sources)."""
    if explicit or (launch_mode in ("plain", "anyhit") and split_ways == 1):
        mix, src, same = find_mix(cfg_name, explicit)
        return ((mix or {}).get("valu_busy_frac"), (mix or {}).get("wave_time_split"), src, same)
    if launch_mode == "spec":
        name = f"c3_share{split_ways}"
        got = {}
        for k in ("spec", "fan"):
            cands = sorted((REPO / "profiles").glob(f"r0*/pmc_mix_{k}_n{split_ways}*.json"),
                           key=lambda q: (q.parent.name, q.name), reverse=True)
            g = _by_sha(cands, lambda c: load_json(str(c), name))
            if g:
                got[k] = (g[0].get("valu_busy_frac"), g[0].get("wave_time_split"), _rel(g[1]), g[2])
        if len(got) == 2:
            return ({k: v[0] for k, v in got.items()}, {k: v[1] for k, v in got.items()},
                    {k: v[2] for k, v in got.items()}, all(v[3] for v in got.values()))
    return None, None, None, None


def sky_pixels(pt, _lib) -> int:
    """Pixels of this context proven to miss every primitive (iqpt_sky_kernel's; 0 when the path is off)."""
    import ctypes as C
    lb = _lib.load()
    lb.iqpt_debug_sky_info.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
    n, t = C.c_uint32(0), C.c_uint32(0)
    _lib.check(lb.iqpt_debug_sky_info(pt.handle, C.byref(n), C.byref(t)), "iqpt_debug_sky_info")
    return int(n.value)


def roofline(cfg, args, world, rays_per_launch, kern_avg_ms, launch_mode: str, split_ways: int, spp: int,
             npix_owned: int, certain_ray_frac: float) -> dict:
    """The dominant kernel against the FP32 vector (VALU) peak.

    C1/C2/C3: algorithmic FLOPs F_ray = 52 T + 19 S per ray (the reference's brute-force
    closest hit) x rays of one launch / the launch's HIP-event time. C4/C5: the BVH and the tile masks
    skip almost all of the brute-force tests, so the work is priced from EXECUTED tests per ray
    (tools/work_counters.py: node tests, leaf Möller–Trumbore tests, sphere tests, from the kOptStats
    counters) when --work-json has them; the brute-force rate is kept as "reference_equivalent"."""
    f_ray = cfg.flops_per_ray
    t = kern_avg_ms * 1e-3
    ref_tflops = f_ray * rays_per_launch / t / 1e12 if t > 0 else 0.0
    # PMC bytes only for the launch shape they were measured on (one GPU's full frame at this spp); the
    # algorithmic bytes (84 B per owned pixel per launch) for every line, rank 0's share at N > 1
    pmc, pmc_src, pmc_same = (find_pmc(cfg.name, spp, args.pmc_json) if world == 1 and not args.share_of
                              else (None, "N > 1: per-rank PMC not collected", None))
    traffic = pmc.get("hbm_bytes_per_launch") if pmc else None
    busy, wsplit, mix_src, mix_same = mix_for_launch(cfg.name, launch_mode, split_ways, args.pmc_mix_json)
    work_path, work_why = (args.work_json, None) if args.work_json else newest_work(cfg.name)
    work = load_json(work_path, cfg.name) if work_path else None
    out = {"bound": "valu", "unit": "TFLOP/s", "peak": FP32_PEAK_TFLOPS,
           "kernel": LAUNCH_KERNELS.get(launch_mode, launch_mode), "launch_mode": launch_mode,
           "kernel_avg_ms": round(kern_avg_ms, 4), "traffic": traffic,
           "valu_busy_frac": busy, "wave_time_split": wsplit, "mix_source": mix_src,
           # whether the PMC profiles were taken on these kernel sources (their kernel_sha16 = the build's)
           "traffic_same_kernel_sources": pmc_same, "mix_same_kernel_sources": mix_same}
    ex = work["flops_per_ray"] * rays_per_launch / t / 1e12 if (work and work.get("flops_per_ray") and t > 0) else None
    if work_why:
        out["executed_work"] = {"missing": work_why}
    if ex is not None and ref_tflops > FP32_PEAK_TFLOPS:
        out.update(achieved=round(ex, 4), frac=round(ex / FP32_PEAK_TFLOPS, 5),
                   flops_per_ray=work["flops_per_ray"], work_basis="executed tests per ray (" + Path(work_path).name + ")",
                   reference_equivalent={"achieved": round(ref_tflops, 2), "flops_per_ray": f_ray,
                                         "frac": round(ref_tflops / FP32_PEAK_TFLOPS, 4)})
    elif ref_tflops <= FP32_PEAK_TFLOPS:
        out.update(achieved=round(ref_tflops, 4), frac=round(ref_tflops / FP32_PEAK_TFLOPS, 5),
                   flops_per_ray=f_ray, work_basis="algorithmic F_ray = 52 T + 19 S (SURVEY.md §8d)")
        if ex is not None:
            # the tests the kernel actually executes (the tile masks skip most of the brute-force ones)
            out["executed_work"] = {"achieved": round(ex, 4), "frac": round(ex / FP32_PEAK_TFLOPS, 5),
                                    "flops_per_ray": work["flops_per_ray"], "per_ray": work.get("per_ray"),
                                    "source": str(Path(work_path).resolve().relative_to(REPO)),
                                    "kernel_sha16": work.get("kernel_sha16")}
    else:
        # the brute-force price exceeds the peak: the kernel skips that work, so it is no roofline
        out.update(achieved=None, frac=None, flops_per_ray=None,
                   work_basis="none: run tools/work_counters.py for the executed-work price",
                   reference_equivalent={"achieved": round(ref_tflops, 2), "flops_per_ray": f_ray})
    # the counted rays include the camera rays of certain-hit and certain-miss (sky) pixels, resolved by a
    # per-pixel proof instead of per-ray tests: the rate of rays that ran a per-ray closest-hit test
    if t > 0:
        out["traced_rays_per_launch"] = round(rays_per_launch * (1.0 - certain_ray_frac))
        out["traced_rays_per_s"] = round(rays_per_launch * (1.0 - certain_ray_frac) / t, 1)
    if t > 0:
        alg = BYTES_PER_PIXEL_LAUNCH * npix_owned
        out["hbm"] = {"achieved": round(alg / t / 1e9, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                      "frac": round(alg / t / 1e9 / HBM_PEAK_GBPS, 6), "basis": "algorithmic",
                      "bytes_per_launch": alg, "pixels_per_launch": npix_owned}
        if traffic:
            out["hbm"].update(pmc_bytes_per_launch=round(traffic), pmc_achieved=round(traffic / t / 1e9, 2),
                              pmc_frac=round(traffic / t / 1e9 / HBM_PEAK_GBPS, 6), pmc_source=pmc_src)
        else:
            out["hbm"]["pmc_source"] = None
            out["hbm"]["pmc_missing"] = pmc_src
    out["note"] = ("achieved = FLOPs per launch / kernel_avg_ms (the HIP-event span of the timed launches / their "
                   "number: overlapped launches run two at a time, launch_duration_ms is one launch's own) against the FP32 "
                   "vector peak; the path runs on the VALU, nothing is a dense contraction (no MFMA). traffic: "
                   "PMC HBM bytes per launch (tools/pmc_traffic.py); valu_busy_frac / wave_time_split: PMC "
                   "instruction-mix pass (tools/pmc_mix.py), profiles/.")
    return out


def newest_work(cfg_name: str):
    """The newest executed-work profile of the config (tools/work_counters.py: profiles/r0*/work_<config>*.json)
    taken on THESE kernel sources (its kernel_sha16 equals the build's, iqpt._build.kernel_source_sha16): counts of
    another kernel price work this kernel may not do. Returns (path, None) or (None, why)."""
    from iqpt._build import kernel_source_sha16
    want = kernel_source_sha16()
    cands = sorted((REPO / "profiles").glob(f"r0*/work_{cfg_name}*.json"), key=lambda q: (q.parent.name, q.name),
                   reverse=True)
    seen = []
    for c in cands:
        d = load_json(str(c), cfg_name)
        if d and d.get("kernel_sha16") == want:
            return str(c), None
        if d:
            seen.append(f"{c.relative_to(REPO)} ({d.get('kernel_sha16') or 'no kernel hash'})")
    return None, (f"no executed-work profile of kernel sources {want}: run tools/work_counters.py --config "
                  f"{cfg_name}" + (f"; stale: {', '.join(seen[:3])}" if seen else ""))


def fma_flavour_rmse():
    """How far a contracting (nvcc-default-like) build of the same algorithm sits from the parity target on
    the full C2 frame (tools/fp_flavours.py): the size of the unpinned part."""
    try:
        d = json.loads((REPO / "profiles" / "r02" / "fp_flavours.json").read_text())
        return d["cases"]["c2_full"]["FMA_vs_B"]["rmse"]
    except (OSError, ValueError, KeyError):
        return None


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    # The per-step gather's stream waits must not share a hardware queue with a render stream: with HIP's
    # 4 queues per process the gather (torch / RCCL stream) and the context's stream land on one queue, and
    # the gather's wait for launch k + 1's frame copy then holds launch k + 2 behind launch k + 1 (profiles/
    # r02/c3_share2_gather_kernel_trace.csv). 8 queues give every stream its own: N = 2 share -10 %
    # (profiles/r02/ab_hw_queues.json). Set before anything initialises HIP.
    strong_gather = (int(os.environ.get("WORLD_SIZE", "1")) > 1 or args.self_gather) and args.scaling != "weak"
    if strong_gather:
        os.environ["GPU_MAX_HW_QUEUES"] = "8"

    import numpy as np
    import torch
    import torch.distributed as dist

    import iqpt
    from iqpt import _lib
    from iqpt import dist as iqdist
    if args.lib:
        _lib.LIB_PATH = Path(args.lib).resolve()
    from iqpt.scene import CONFIGS, Scene, make_camera, packet_stats

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # Rehearsal of the multi-rank path on a 1-GPU box: every rank on device 0 and the collectives over
    # gloo through host memory (RCCL refuses two ranks on one GPU). The driver's runs use nccl.
    device = 0 if args.one_device else local_rank
    torch.cuda.set_device(device)
    use_pg = world > 1 or args.self_gather
    if use_pg:
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            os.environ.setdefault("RANK", "0")
        # torch.distributed only for the rendezvous, the barriers and the post-timing reductions (host, gloo);
        # the data path's collective — the per-step frame gather over RCCL / xGMI — is libiqpt's own
        # communicator (iqpt_comm_init / iqpt_gather_frame_async). --backend gloo keeps a host
        # gather through torch for the one-device multi-rank rehearsal (RCCL refuses two ranks on one GPU).
        dist.init_process_group("gloo", world_size=world, rank=rank)
    n_ranks_seen = dist.get_world_size() if use_pg else 1

    def barrier():
        if world > 1:
            dist.barrier()

    cfg = CONFIGS[args.config]
    spp_step = args.spp or cfg.spp
    scene = Scene()
    scene.add_preset(cfg.preset)
    pk = scene.build_packet()
    stats = packet_stats(pk)
    cam = make_camera(cfg.width, cfg.height)
    weak = args.scaling == "weak"
    # weak: the whole frame per rank, RNG streams of seed 1984 + rank; strong: cyclic rows of one frame
    part_rank, part_world = (0, 1) if weak else (rank, world)
    if args.share_of:
        if world != 1 or weak:
            raise SystemExit("--share-of is a one-rank strong-scaling rehearsal")
        part_world = args.share_of
    seed = iqpt.DEFAULT_SEED + (rank if weak else 0)
    ps = iqdist.pixel_set_for_rank(cfg.width, cfg.height, part_rank, part_world)
    setup = {}
    t0 = time.perf_counter()
    pt = iqpt.PathTracer(cfg.width, cfg.height, pixels=ps, seed=seed, max_depth=cfg.max_depth, device=device)
    setup["create_and_rng_init_ms"] = (time.perf_counter() - t0) * 1e3
    pt.set_split({"auto": _lib.SPLIT_AUTO, "on": _lib.SPLIT_ON, "off": _lib.SPLIT_OFF,
                  "spec": _lib.SPLIT_SPEC}[args.split])
    if args.kernel_options:
        import ctypes as C
        _lib.load().iqpt_debug_set_kernel_options.argtypes = [C.c_void_p, C.c_int]
        _lib.check(_lib.load().iqpt_debug_set_kernel_options(pt.handle, args.kernel_options),
                   "iqpt_debug_set_kernel_options")
    pt.set_overlap(_lib.OVERLAP_AUTO if args.overlap == "auto" else _lib.OVERLAP_OFF)
    if args.sky_order is not None:
        import ctypes as C
        lb = _lib.load()
        lb.iqpt_debug_set_sky_order.argtypes = [C.c_void_p, C.c_int]
        _lib.check(lb.iqpt_debug_set_sky_order(pt._h, 1 if args.sky_order == "behind" else 0),
                   "iqpt_debug_set_sky_order")
    if args.no_kernel_timing:
        import ctypes as C
        lb = _lib.load()
        lb.iqpt_debug_set_timing.argtypes = [C.c_void_p, C.c_int]
        _lib.check(lb.iqpt_debug_set_timing(pt._h, 0), "iqpt_debug_set_timing")
    if args.certain == "off":
        import ctypes as C
        lb = _lib.load()
        lb.iqpt_debug_set_certain.argtypes = [C.c_void_p, C.c_int]
        _lib.check(lb.iqpt_debug_set_certain(pt._h, 0), "iqpt_debug_set_certain")
    if args.sky == "off":
        import ctypes as C
        lb = _lib.load()
        lb.iqpt_debug_set_sky.argtypes = [C.c_void_p, C.c_int]
        _lib.check(lb.iqpt_debug_set_sky(pt._h, 0), "iqpt_debug_set_sky")
    if args.two_ray is not None:
        import ctypes as C
        lb = _lib.load()
        lb.iqpt_debug_set_two_ray.argtypes = [C.c_void_p, C.c_int]
        _lib.check(lb.iqpt_debug_set_two_ray(pt._h, args.two_ray), "iqpt_debug_set_two_ray")
    if args.anyhit is not None:
        import ctypes as C
        lb = _lib.load()
        lb.iqpt_debug_set_anyhit.argtypes = [C.c_void_p, C.c_int]
        _lib.check(lb.iqpt_debug_set_anyhit(pt._h, args.anyhit), "iqpt_debug_set_anyhit")
    if args.pixel_masks is not None:
        import ctypes as C
        lb = _lib.load()
        lb.iqpt_debug_set_pixel_masks.argtypes = [C.c_void_p, C.c_int]
        _lib.check(lb.iqpt_debug_set_pixel_masks(pt._h, args.pixel_masks), "iqpt_debug_set_pixel_masks")
    if args.stream_refill is not None:
        import ctypes as C
        lb = _lib.load()
        lb.iqpt_debug_set_stream_refill.argtypes = [C.c_void_p, C.c_uint32]
        _lib.check(lb.iqpt_debug_set_stream_refill(pt._h, args.stream_refill), "iqpt_debug_set_stream_refill")
    if args.stream_xcd is not None:
        import ctypes as C
        lb = _lib.load()
        lb.iqpt_debug_set_stream_xcd.argtypes = [C.c_void_p, C.c_int]
        _lib.check(lb.iqpt_debug_set_stream_xcd(pt._h, args.stream_xcd), "iqpt_debug_set_stream_xcd")
    if args.resident_refill is not None:
        import ctypes as C
        lb = _lib.load()
        lb.iqpt_debug_set_resident_refill.argtypes = [C.c_void_p, C.c_uint32]
        _lib.check(lb.iqpt_debug_set_resident_refill(pt._h, args.resident_refill), "iqpt_debug_set_resident_refill")
    if args.spec_margin is not None:
        import ctypes as C
        lb = _lib.load()
        lb.iqpt_debug_set_spec.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
        _lib.check(lb.iqpt_debug_set_spec(pt._h, 0, args.spec_margin), "iqpt_debug_set_spec")
    if args.spec_parity is not None:
        import ctypes as C
        lb = _lib.load()
        lb.iqpt_debug_set_spec_parity.argtypes = [C.c_void_p, C.c_uint32]
        _lib.check(lb.iqpt_debug_set_spec_parity(pt._h, int(round(args.spec_parity * 256))), "iqpt_debug_set_spec_parity")
    pt.set_camera(cam)
    t0 = time.perf_counter()
    pt.upload_packet(pk)
    setup["upload_relayout_bvh_ms"] = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    pt.prepare()
    setup["tile_masks_order_split_ms"] = (time.perf_counter() - t0) * 1e3

    on_gpu = args.backend == "nccl"
    tdev = "cuda" if on_gpu else "cpu"
    max_px = iqdist.max_rows(cfg.height, part_world) * cfg.width
    strong_multi = (world > 1 or args.self_gather) and not weak
    words = 4 if args.gather == "accum" else 1
    dtype = torch.float32 if args.gather == "accum" else torch.int32
    # nccl: libiqpt's RCCL communicator gathers the BGRA8 frame (or the accumulators) to rank 0 and assembles
    # it there on the device (W x H, row-major); gloo: the host gather below
    lib_gather = strong_multi and on_gpu
    if lib_gather:
        uid = [iqpt.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        if args.gather_ctas is not None or args.gather_prio is not None or args.gather_skip:
            import ctypes as C
            lb = _lib.load()
            lb.iqpt_debug_set_gather.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int]
            _lib.check(lb.iqpt_debug_set_gather(pt._h, 2 if args.gather_ctas is None else args.gather_ctas,
                                                0 if args.gather_prio is None else args.gather_prio,
                                                args.gather_skip), "iqpt_debug_set_gather")
        pt.comm_init(rank, world, uid[0])
    frame_dev = (torch.zeros((cfg.width * cfg.height, words), dtype=dtype, device="cuda")
                 if lib_gather and rank == 0 else None)
    buf = torch.zeros((max_px, words), dtype=dtype, device=tdev) if strong_multi and not lib_gather else None
    gather_list = ([torch.empty_like(buf) for _ in range(world)]
                   if (strong_multi and not lib_gather and rank == 0) else None)
    assembled = None

    def fetch(dst, what):
        n = dst.numel() * 4
        if on_gpu:
            (pt.copy_accum_device if what == "accum" else pt.copy_frame_device)(dst.data_ptr(), n)
        else:
            lin_host, bgra_host = pt.read()
            src = lin_host if what == "accum" else bgra_host.view(np.int32)
            dst[: src.shape[0]] = torch.from_numpy(np.ascontiguousarray(src).reshape(src.shape[0], -1))

    def deinterleave(parts, channels):
        # rank r holds rows r, r + N, ...: [N, rows, W, c] -> [rows, N, W, c] -> the first H rows
        st = torch.stack(parts).view(world, -1, cfg.width, channels)
        return st.transpose(0, 1).reshape(-1, cfg.width, channels)[: cfg.height]

    # Stream-ordered gather (nccl, BGRA frame, libiqpt): the copy of the step's frame is enqueued behind its
    # render (on the launch's own stream: overlapped and pipelined launches keep overlapping), the RCCL
    # gather and rank 0's assembly on the communicator's stream behind the copy; no host synchronisation
    # inside the timed steps, and the gather of step k runs while step k + 1 renders.
    stream_gather = lib_gather and args.gather == "frame" and not args.gather_sync

    host = {"render": 0.0, "gather": 0.0}          # host time inside the library's calls (timed steps)

    def step():
        nonlocal assembled
        h0 = time.perf_counter()
        pt.render(spp_step)
        h1 = time.perf_counter()
        host["render"] += h1 - h0
        if stream_gather:
            pt.gather_frame_async(0, frame_dev.data_ptr() if rank == 0 else 0,
                                  frame_dev.numel() * 4 if rank == 0 else 0)
            host["gather"] += time.perf_counter() - h1
            assembled = frame_dev
        elif lib_gather:
            # --gather-sync / --gather accum: the blocking form
            if args.gather == "accum":
                pt.gather_accum(0, frame_dev.data_ptr() if rank == 0 else 0, frame_dev.numel() * 4 if rank == 0 else 0)
            else:
                pt.gather_frame_async(0, frame_dev.data_ptr() if rank == 0 else 0,
                                      frame_dev.numel() * 4 if rank == 0 else 0)
                pt.sync()
            assembled = frame_dev
        elif strong_multi:
            fetch(buf, args.gather)
            dist.gather(buf, gather_list, dst=0)
            if rank == 0:
                assembled = deinterleave(gather_list, words)

    # warmup (the first frame is also checked against the oracle). The frame is read here, the oracle
    # runs after the timed steps: seconds of host work with the GPU idle just before the timed region
    # cost ~40 us per step outside the kernels in the 20-step driver runs (r03 run 52: 1.016 ms per step
    # against 0.987 without the check, at the same kernel span)
    verify = None
    first_lin = None
    for i in range(max(1, args.warmup)):
        step()
        if i == 0 and args.verify_rows > 0:
            first_lin = pt.read()[0]
    torch.cuda.synchronize()
    barrier()
    rays0 = pt.rays()
    pt.kernel_time()                                   # discard warmup timings
    torch.cuda.synchronize()
    barrier()
    host["render"] = host["gather"] = 0.0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    pt.sync()
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    rays = pt.rays() - rays0
    kern_ms, launches = pt.kernel_time()
    # overlapped launches run two at a time: the event span of the timed launches / their
    # number is the kernel time per launch that the throughput sees; each launch's own duration is longer
    kern_span_ms = pt.kernel_span()
    gather_ms, gathers = pt.comm_time() if lib_gather else (0.0, 0)
    launch_mode = pt.launch_mode()
    import ctypes as C
    _lb = _lib.load()
    _lb.iqpt_debug_last_options.argtypes = [C.c_void_p, C.POINTER(C.c_int)]
    _o = C.c_int(0)
    _lib.check(_lb.iqpt_debug_last_options(pt.handle, C.byref(_o)), "iqpt_debug_last_options")
    last_opt = _o.value & ~((1 << 30) | (1 << 29))    # the render-kernel option set of the last launch
    xcd_lists = bool(_o.value & (1 << 30))             # ... whose tiles were dealt to per-XCD lists
    if _o.value >= 0 and _o.value & (1 << 29):         # ... rendered by iqpt_anyhit_kernel instead (C4)
        launch_mode = "anyhit"
    certain_px = certain_pixels(pt, _lib) if args.certain != "off" else 0
    sky_px = sky_pixels(pt, _lib) if (args.certain != "off" and args.sky != "off") else 0

    # the last step's gathered frame: rank 0's own rows of it must be its own frame (checks the gather path;
    # libiqpt's assembly puts them at rows 0, S, 2S, ... of the W x H frame, S = the split's ways)
    gather_check = None
    if strong_multi and rank == 0 and assembled is not None:
        torch.cuda.synchronize()
        lin_own, bgra_own = pt.read()
        own = (lin_own.view(np.int32) if words == 4 else bgra_own.view(np.int32)).reshape(-1, cfg.width * words)
        step_rows = part_world if lib_gather else world
        got = assembled.reshape(-1, cfg.width * words)[0::step_rows][: own.shape[0]].cpu().numpy().view(np.int32)
        gather_check = bool(own.shape == got.shape and np.array_equal(own, got))

    # after timing: the float frame on rank 0 (strong: the gathered accumulators assembled, bit-identical to
    # one GPU's frame; weak: the N independent estimates averaged)
    frame = None
    if world > 1 and lib_gather:
        acc = torch.zeros((cfg.width * cfg.height, 4), dtype=torch.float32, device="cuda") if rank == 0 else None
        pt.gather_accum(0, acc.data_ptr() if rank == 0 else 0, acc.numel() * 4 if rank == 0 else 0)
        frame = acc
    elif world > 1:
        acc = torch.zeros((max_px, 4), dtype=torch.float32, device=tdev)
        fetch(acc, "accum")
        if weak:
            dist.reduce(acc, dst=0, op=dist.ReduceOp.SUM)
            if rank == 0:
                frame = (acc / float(world))[: cfg.width * cfg.height]
        else:
            parts = [torch.empty_like(acc) for _ in range(world)] if rank == 0 else None
            dist.gather(acc, parts, dst=0)
            if rank == 0:
                frame = deinterleave(parts, 4).reshape(-1, 4)

    if first_lin is not None:
        verify = verify_vs_oracle(cfg, pk, cam, first_lin, part_rank, part_world, min(args.verify_rows, ps.nrows),
                                  seed=seed, spp=spp_step)
        first_lin = None

    vals = torch.tensor([elapsed, float(rays), kern_span_ms / max(1, launches), verify["rmse"] if verify else 0.0,
                         verify["bitexact_frac"] if verify else 1.0], dtype=torch.float64)
    # per rank (N > 1 lines): the render span per launch, the step, the gathers' own time per step on the
    # communicator stream (transfer + waiting for slower ranks), and the step time outside the render span
    mine = {"rank": rank, "render_span_ms": round(kern_span_ms / max(1, launches), 4),
            "step_ms": round(elapsed / args.steps * 1e3, 4),
            "gather_ms": round(gather_ms / gathers, 4) if gathers else None,
            "outside_render_ms": round(elapsed / args.steps * 1e3 - kern_span_ms / max(1, launches), 4),
            # the host's time per step inside iqpt_render / iqpt_gather_frame_async: a host slower than the GPU
            # leaves the GPU idle between launches
            "host_render_ms": round(host["render"] / args.steps * 1e3, 4),
            "host_gather_ms": round(host["gather"] / args.steps * 1e3, 4),
            "bitexact_frac_vs_oracle": verify["bitexact_frac"] if verify else None}
    per_rank = [None] * world if world > 1 else [mine]
    if world > 1:
        dist.all_gather_object(per_rank, mine)
    if world > 1:
        mx = vals[[0, 2, 3]].clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        tot = vals[1:2].clone()
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        mn = vals[4:5].clone()
        dist.all_reduce(mn, op=dist.ReduceOp.MIN)
        elapsed, kern_avg_ms, rmse_v = mx.tolist()
        total_rays, bitexact = tot.item(), mn.item()
    else:
        total_rays, kern_avg_ms = float(rays), kern_span_ms / max(1, launches)
        rmse_v, bitexact = (verify["rmse"], verify["bitexact_frac"]) if verify else (None, None)

    npix_owned = (ps.x1 - ps.x0) * ps.nrows
    if rank == 0:
        mrays = total_rays / elapsed / 1e6
        rays_per_launch = float(rays) / max(1, args.steps)           # rank 0's kernel
        samples = cfg.width * cfg.height * spp_step * args.steps * (world if weak else 1)
        gathered = "BGRA8 frame" if args.gather == "frame" else "float4 accumulators"
        out = {
            "metric": "Mrays/sec at 1920x1080 8-bounce; per-pixel RMSE vs reference",
            # "RMSE vs reference" is measured against the oracle restatement (parity_basis below)
            "value": round(mrays, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak" if weak else "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": ("synthetic (procedural scene of SURVEY.md §8d, seed 1984"
                     + (", rank r: seed 1984+r)" if weak and world > 1 else ")")),
            "config": {"workload": f"{cfg.name}:{cfg.preset}" + ("" if world == 1 or weak else " (C3 row-tiled)"),
                       "width": cfg.width, "height": cfg.height,
                       "spp_per_step": spp_step, "max_depth": cfg.max_depth, "triangles": stats["triangles"],
                       "spheres": stats["spheres"],
                       "partition": (f"full frame per rank x{world} (seed 1984+rank)" if weak
                                     else (f"cyclic rows x{world}" if world > 1 else
                                           (f"rank 0's rows of a cyclic x{args.share_of} split (one-GPU share "
                                            "rehearsal)" if args.share_of else "full frame"))),
                       "collective": ("none" if not (strong_multi or world > 1) else
                                      ("none in the timed region; one reduce of the accumulators after it"
                                       if weak else f"gather of the {gathered} to rank 0 every step")
                                      + (" (RCCL ncclGather inside libiqpt: iqpt_gather_frame_async)" if lib_gather
                                         else " (gloo via host, rehearsal)")),
                       "split": args.split, "overlap": args.overlap, "certain": args.certain, "sky": args.sky,
                       "launch_mode": launch_mode,
                       # the plain kernel's option bits of the last launch (iqpt_internal.hpp kOpt*): for streamed
                       # scenes bit 12 (kOptBvhPrimary) says whether camera rays took the BVH or the tile lists
                       "kernel_option_bits": hex(last_opt),
                       "xcd_tile_lists": xcd_lists,
                       **({"kernel_options": args.kernel_options} if args.kernel_options else {}),
                       **({"spec_parity": args.spec_parity} if args.spec_parity is not None else {}),
                       **({"spec_margin": args.spec_margin} if args.spec_margin is not None else {}),
                       **({"anyhit": args.anyhit} if args.anyhit is not None else {}),
                       **({"pixel_masks": args.pixel_masks} if args.pixel_masks is not None else {}),
                       **({"stream_refill": args.stream_refill} if args.stream_refill is not None else {}),
                       **({"resident_refill": args.resident_refill} if args.resident_refill is not None else {}),
                       **({"stream_xcd": args.stream_xcd} if args.stream_xcd is not None else {}),
                       **({"warmup_note": "W < 5: launches that time the camera-ray paths fall in the timed region"}
                          if args.config in STREAMED_CONFIGS and args.warmup < 5 else {})},
            "n_ranks_seen": n_ranks_seen,
            "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
            # the libiqpt that ran (its ABI; an A/B --lib may be an older build)
            "lib": {"path": str(_lib.LIB_PATH.name) if not args.lib else args.lib, "abi": _lib.LOADED_ABI},
            **({"gather": "stream-ordered" if stream_gather else "blocking", "gather_check": gather_check}
               if strong_multi else {}),
            "msamples_per_s": round(samples / elapsed / 1e6, 3),
            "rays_per_sample": round(total_rays / samples, 5),
            # value counts the closest-hit queries the reference performs for the same image; the camera rays
            # of certain pixels are among them but resolved by one interval proof per pixel
            # (every ray of the pixel's jitter square hits an emissive triangle first) instead of per-ray tests
            "certain_pixels": {"pixels": certain_px, "frac_of_owned_pixels": round(certain_px / max(1, npix_owned), 5),
                               "frac_of_rays_counted": round(certain_px * spp_step * args.steps / max(1.0, float(rays)), 5),
                               "note": "rank 0's pixels whose camera rays are proven (iq_interval.h tri_certain) to end "
                                       "on an emissive triangle: their samples take the two camera draws and fold "
                                       "the clamped (1, 1, 1) without a per-ray intersection test; bit-identical "
                                       "results (tests/test_gpu_certain.py)"},
            # pixels proven (iq_interval.h) to miss every primitive: their samples are one camera ray each, the sky
            # gradient, rendered by iqpt_sky_kernel without an intersection test
            "sky_pixels": {"pixels": sky_px, "frac_of_owned_pixels": round(sky_px / max(1, npix_owned), 5),
                           "frac_of_rays_counted": round(sky_px * spp_step * args.steps / max(1.0, float(rays)), 5)},
            "rmse_vs_oracle": rmse_v,
            "bitexact_frac_vs_oracle": bitexact,
            "setup_ms": {k: round(v, 2) for k, v in setup.items()},
            "parity_basis": ("bit-exact vs the CPU oracle (oracle/iqpt_oracle.c: the reference restated with "
                             "FMA contraction off and shared iq_fp.h transcendentals); unpinned vs the nvcc/cuRAND "
                             "reference binary, which cannot be built here"),
            "fma_flavour_rmse_c2": fma_flavour_rmse(),
            "roofline": roofline(cfg, args, world, rays_per_launch, kern_avg_ms, launch_mode, part_world, spp_step,
                                 npix_owned, (certain_px + sky_px) * spp_step * args.steps / max(1.0, float(rays))),
        }
        if strong_multi or world > 1:
            out["per_rank"] = per_rank
        out["roofline"]["launch_duration_ms"] = round(kern_ms / max(1, launches), 4)
        out["roofline"]["overlapped_launches"] = bool(kern_span_ms < 0.98 * kern_ms)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(cfg, pk, cam, args.cpu_seconds)
        if args.save_frame:
            if frame is None:
                frame = torch.from_numpy(pt.read()[0])
            np.save(args.save_frame, frame.cpu().numpy())
        print(json.dumps(out), flush=True)
    pt.close()
    if use_pg:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
