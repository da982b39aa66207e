#!/usr/bin/env python3
"""Throughput bench: points/s of one training step (forward + masked one-hot CE +
backward + gradient all-reduce + Adam step) on 4096-point S3DIS-like blocks.

Headline (BASELINE.json metric "points/sec fwd+bwd, 4096-pt S3DIS blocks,
PointNet++/DGCNN @1/2/4/8 GPU"): `value` is PointNet++ SSG, batch 32 per GPU,
4096 points (configs[1]); the same JSON line carries the DGCNN EdgeConv half of the
metric (configs[2]: DGCNN-colour k=20, batch 32 per GPU) as `secondary`, timed the
same way in the same process.  fp32, synthetic blocks resident in HBM before timing.

Multi-GPU: one process per GPU, data-parallel, RCCL all-reduce of the flat gradient
buffer, fixed per-GPU batch ("weak" scaling).  `--gpus N` either runs under an
external launcher (torchrun sets WORLD_SIZE, which must equal N) or, without one,
spawns the N rank processes itself before touching the GPU.

Also reported on the same JSON line, per workload:
  roofline      -- the dominant HIP kernel (the engine GEMM variant with the largest
                   time in one probed step): its algorithmic flops and bytes per launch
                   over its IN-STEP launch time (HIP events on the stream it runs on,
                   the step enqueued behind a spin so the GPU runs it back to back as
                   in a GPU-bound step), against the fp32 MFMA peak or the HBM peak by
                   its arithmetic intensity;
  cpu_baseline  -- the CPU oracle (oracle/ref_ops.py, the reference algorithm restated
                   on PyTorch-CPU) on the same batch size, median step time, in a
                   subprocess with no GPU visible, rank 0 at N=1 only.
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import socket
import statistics
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.join(REPO, '3d-semantic-segmentation-benchmark_amd')
for _p in (REPO, PKG_ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

# key: (class name, ctor, input kind, default per-GPU batch, default points, BASELINE config)
WORKLOADS = {
    'pointnetpp': ('PointNetpp', lambda m: m.PointNetpp(14), 'points', 32, 4096,
                   'configs[1] PointNet++ SSG seg, 4096 pts, batch 32/GPU'),
    'dgcnn': ('DGCNNWithColor', lambda m: m.DGCNNWithColor(num_classes=14, k=20), 'chfirst6', 32, 4096,
              'configs[2] DGCNN EdgeConv seg (colour), 4096 pts, k=20, batch 32/GPU'),
    'pointnetpp_msg': ('PointNetppMSG', lambda m: m.PointNetppMSG(14), 'points', 32, 4096,
                       'configs[3] PointNet++ MSG seg, 4096 pts, batch 32/GPU (256 on 8 GPUs)'),
    'pointnext': ('PointNeXt', lambda m: m.PointNeXt(14), 'points', 16, 24576,
                  'configs[4] PointNeXt-B seg, 24576 pts, batch 16/GPU (128 on 8 GPUs)'),
    'pointnet': ('PointNetSeg', lambda m: m.PointNetSeg(part_classes=14), 'points', 32, 4096,
                 'PointNet seg, 4096 pts, batch 32/GPU (configs[0] model on the GPU)'),
}
METRIC = 'points/sec fwd+bwd, 4096-pt S3DIS blocks, PointNet++/DGCNN @1/2/4/8 GPU'
# CPU baseline batch per workload: a bounded sample of the same workload, ~5-6 s per CPU step
CPU_BATCH = {'pointnetpp': 32, 'dgcnn': 8, 'pointnetpp_msg': 16, 'pointnext': 2, 'pointnet': 16}
HBM_PEAK_GBS = 8000.0           # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_PEAK_TFLOPS = 157.3        # fp32 MFMA dense (= fp32 vector) peak
RIDGE = FP32_PEAK_TFLOPS * 1e12 / (HBM_PEAK_GBS * 1e9)     # flop / byte
# reference-algorithm fwd+bwd GFLOP per sample (FlopCounterMode on the reference)
# (MSG: the oracle composition, scripts/flops_msg.py -- same method, which reproduces SSG's 5.786)
ALGO_GFLOP_PER_SAMPLE = {('pointnetpp', 4096): 5.786, ('pointnext', 4096): 10.791, ('pointnext', 24576): 19.592,
                         ('dgcnn', 4096): 53.468, ('pointnet', 4096): 24.635, ('pointnetpp_msg', 4096): 8.701}


def model_input(pts, kind):
    if kind == 'chfirst6':
        return pts[:, :, :6].contiguous().transpose(1, 2)   # (B,6,N) view, as harness B passes it
    return pts


def logits_of(out):
    return out[0] if isinstance(out, tuple) else out


def host_cpu_info():
    """(threads this process may use, physical cores of the host from sysfs or None)."""
    aff = len(os.sched_getaffinity(0))
    phys = set()
    try:
        base = '/sys/devices/system/cpu'
        for d in os.listdir(base):
            p = os.path.join(base, d, 'topology', 'core_id')
            if d.startswith('cpu') and d[3:].isdigit() and os.path.exists(p):
                pkg = open(os.path.join(base, d, 'topology', 'physical_package_id')).read().strip()
                phys.add((pkg, open(p).read().strip()))
    except OSError:
        phys = set()
    return aff, (len(phys) or None)


# ----------------------------------------------------------------------------- CPU baseline worker
def cpu_baseline_worker(args):
    import torch
    from oracle import ref_ops as R
    from pcseg.synthetic import make_batch
    torch.set_num_threads(args.cpu_threads)
    name, ctor, kind, _, _, _ = WORKLOADS[args.model]
    model = R.seeded_init_(ctor(R), 0)
    model.train()
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    pts, labels, lengths = make_batch(args.cpu_batch, args.npoints, seed=1000)
    x = model_input(pts, kind)
    lab = labels.float() if kind == 'chfirst6' else labels

    def step():
        opt.zero_grad()
        loss = R.masked_onehot_cross_entropy(logits_of(model(x)), lab, lengths)
        loss.backward()
        opt.step()
    t0 = time.perf_counter()
    step()
    warm = time.perf_counter() - t0
    # timed steps: cpu_steps (>= 5 by default), fewer only past ~cpu_budget seconds, at least 3
    n = max(3, min(args.cpu_steps, int(args.cpu_budget / max(warm, 1e-3))))
    times = []
    for i in range(n):
        t0 = time.perf_counter()
        step()
        times.append(time.perf_counter() - t0)
        # progress on stderr (a silent minute reads as a hang to the GPU box's watchdog)
        print(f'[bench] cpu baseline {name} {torch.get_num_threads()} threads: step {i + 1}/{n} '
              f'{times[-1]:.2f} s', file=sys.stderr, flush=True)
    med = statistics.median(times)
    print(json.dumps({'value': args.cpu_batch * args.npoints / med, 'unit': 'points/s',
                      'cores': torch.get_num_threads(), 'kind': 'port',
                      'sample': f'{name} oracle (PyTorch-CPU restatement of the reference, fp32), batch '
                                f'{args.cpu_batch} x {args.npoints} pts, fwd+CE+bwd+Adam, 1 warm-up + median of '
                                f'{n} steps ({sum(times):.1f} s timed)'}))


def _cpu_run(args, key, batch, npoints, threads):
    env = dict(os.environ, HIP_VISIBLE_DEVICES='', CUDA_VISIBLE_DEVICES='', OMP_NUM_THREADS=str(threads))
    cmd = [sys.executable, os.path.abspath(__file__), '--cpu-baseline-worker', '--model', key,
           '--npoints', str(npoints), '--cpu-batch', str(batch), '--cpu-steps',
           str(args.cpu_steps), '--cpu-threads', str(threads), '--cpu-budget', str(args.cpu_budget)]
    try:
        print(f'[bench] cpu baseline {key} on {threads} threads', file=sys.stderr, flush=True)
        out = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, text=True, timeout=900, check=True).stdout
        return json.loads(out.strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001 -- the baseline is informative, never fatal
        return {'value': None, 'unit': 'points/s', 'cores': threads, 'kind': 'port', 'sample': f'failed: {e}'}


def run_cpu_baseline(args, key, batch, npoints):
    """The oracle on the host's CPU share (16 threads on the GPU box: OMP_NUM_THREADS there) and,
    beside it, on every physical core of the host; >= cpu_steps timed steps each on a bounded
    batch (CPU_BATCH: about 30 s per run)."""
    aff, phys = host_cpu_info()
    share = args.cpu_threads or min(aff, int(os.environ.get('OMP_NUM_THREADS', '16') or 16), 16)
    cb = args.cpu_batch or min(batch, CPU_BATCH.get(key, batch))
    res = _cpu_run(args, key, cb, npoints, share)
    full = min(aff, phys) if phys else aff
    if not args.cpu_threads and full > share:
        res['all_physical_cores'] = _cpu_run(args, key, cb, npoints, full)
    res['host_cpus_visible'] = aff
    res['host_physical_cores'] = phys
    return res


# ----------------------------------------------------------------------------- roofline of the dominant kernel
def _by_round(files):
    """Committed profile files sorted by their round number (r05 < r10), last = newest."""
    import re
    return sorted(files, key=lambda f: (int(m.group(1)) if (m := re.match(r'r(\d+)_', os.path.basename(f)))
                                         else -1, f))


def pmc_traffic(kernel, key, batch, npoints):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary of this workload
    (scripts/gpu_pmc.sh -> profiles/<round>_pmc_<model>_b<B>_n<N>.json; FETCH_SIZE x2 + WRITE_SIZE).
    Not measured in this run: the PMC passes are separate rocprofv3 runs (MI355X_MICROARCH.md)."""
    import glob
    files = _by_round(glob.glob(os.path.join(REPO, 'profiles', f'*_pmc_{key}_b{batch}_n{npoints}.json')))
    if not files:
        return None, None
    table = json.load(open(files[-1]))
    for k, v in table.items():
        if kernel in k:
            return round(v['hbm_bytes_per_launch']), os.path.relpath(files[-1], REPO)
    return None, None


def committed_profile_avg_us(kernel, key):
    """The kernel's average duration in the newest COMMITTED rocprofv3 --stats summary of this
    workload's bench step (profiles/<round>_<model>_rocprof_stats.txt, scripts/prof_summary.py
    format).  Read from the file, not measured in this run: the cross-check of the live HIP-event
    average (the events bracket each launch, so they also count its dispatch latency)."""
    import glob
    files = _by_round(glob.glob(os.path.join(REPO, 'profiles', f'*_{key}_rocprof_stats.txt')))
    if not files:
        return None, None
    for line in open(files[-1]):
        parts = line.split()
        if len(parts) > 5 and parts[1] == 'ms/step' and parts[4] == 'us' and kernel in line:
            return float(parts[3]), os.path.relpath(files[-1], REPO)
    return None, None


def _kernel_entry(name, n, fl, by, sec):
    """Roofline of one kernel from its summed in-step launches."""
    intensity = fl / by if by else float('inf')
    bound = 'mfma' if intensity >= RIDGE else 'hbm'
    tf, gbs = fl / sec / 1e12, by / sec / 1e9
    achieved, peak, unit = (tf, FP32_PEAK_TFLOPS, 'TFLOP/s') if bound == 'mfma' else (gbs, HBM_PEAK_GBS, 'GB/s')
    # fp32 compute on gfx950: the MFMA and the vector ALU share the 157.3 TF peak; the neighbour
    # search kernels (FPS, ball query, 3-NN) are VALU kernels, the engine GEMMs and kNN MFMA ones
    unit_kind = 'valu' if any(k in name for k in ('fps_kernel', 'select_kernel', 'three_nn')) else \
        ('mfma' if any(k in name for k in ('gemm', 'wgrad', 'fused_bwd', 'knn_wave')) else 'memory')
    return {'kernel': name, 'bound': bound, 'achieved': round(achieved, 2), 'peak': peak, 'unit': unit,
            'frac': round(achieved / peak, 4), 'compute_unit': unit_kind, 'launches_per_step': n,
            'avg_launch_us': round(sec / n * 1e6, 2), 'in_step_ms': round(sec * 1e3, 3),
            'algo_flops_per_launch': round(fl / n), 'algo_bytes_per_launch': round(by / n),
            'arith_intensity_flop_per_byte': round(intensity, 2) if by else None,
            'achieved_tflops': round(tf, 2), 'frac_of_fp32_peak': round(tf / FP32_PEAK_TFLOPS, 4),
            'achieved_hbm_gbs': round(gbs, 1), 'frac_of_hbm_peak': round(gbs / HBM_PEAK_GBS, 4)}


def concurrent_mfma(tl, name, main):
    """The MFMA work done on the whole GPU while the dominant kernel runs: its own flops plus the
    flops of the side-stream MFMA launches (the wgrad lane's weight gradients of the same layers)
    pro rata of their overlap with its launches, over its summed launch time.  The in-step
    data-gradient GEMMs share the CUs with those weight gradients, so their own fraction
    understates how busy the matrix cores are."""
    mine = [(t0, t1, fl) for n, fl, sh, t0, t1 in tl if n == name and sh == main]
    others = [(t0, t1, fl, n) for n, fl, sh, t0, t1 in tl
              if sh != main and any(k in n for k in ('gemm', 'wgrad', 'fused_bwd', 'knn_wave'))]
    if not mine:
        return None
    busy = sum(t1 - t0 for t0, t1, _ in mine)
    own = sum(fl for _, _, fl in mine)
    side, names = 0.0, set()
    for a0, a1, _ in mine:
        for b0, b1, fl, n in others:
            ov = min(a1, b1) - max(a0, b0)
            if ov > 0 and b1 > b0:
                side += fl * ov / (b1 - b0)
                names.add(n)
    tf = (own + side) / max(busy, 1e-12) / 1e12
    return {'tflops': round(tf, 2), 'frac_of_fp32_peak': round(tf / FP32_PEAK_TFLOPS, 4),
            'own_tflops': round(own / max(busy, 1e-12) / 1e12, 2),
            'side_gflop_overlapped': round(side / 1e9, 3), 'side_kernels': sorted(names),
            'note': 'dominant kernel flops + side-stream MFMA flops pro rata of overlap, over the dominant '
                    'kernel\'s summed launch time (probe events)'}


def kernel_roofline(step, dev, key, batch, npoints, replay=False):
    """One more training step with every probed HIP launch -- engine GEMMs, FPS, ball query,
    3-NN, kNN, gathers, inverse maps, EdgeConv -- bracketed by HIP events on its own stream
    (csrc/probe.cpp).  The step is enqueued behind a 50 ms spin on the main stream, so the GPU
    runs the whole step back to back (as it does in the GPU-bound timed loop) and the event
    pairs time the kernels, not host-enqueue gaps.  The dominant kernel is the one with the
    largest summed in-step time on the step's own stream -- the critical path: the side
    streams (the next step's geometry, the wgrad lane) run under it; `achieved` = its
    algorithmic flops or bytes (per-launch models in DESIGN.md section 3) over that time.  Also
    returned: the largest side-stream kernel (`largest_side_stream_kernel`, e.g. PointNet++'s
    prefetched FPS), the top kernels over all streams, and the flops the probed launches
    execute per sample (`executed_gflop_per_step`)."""
    import torch
    from pcseg.engine import KernelProbe
    from pcseg._lib import call, stream_ptr
    torch.cuda.synchronize(dev)
    main = stream_ptr(dev)
    call('pcs_spin', 50000, main)
    with KernelProbe() as kp:
        step()
    summ = kp.summary()
    crit = kp.summary(stream=int(main))
    side = kp.summary(stream=int(main), exclude=True)
    torch.cuda.synchronize(dev)
    ranked = sorted(summ.items(), key=lambda kv: -kv[1][3])
    name, (n, fl, by, sec) = sorted(crit.items(), key=lambda kv: -kv[1][3])[0]
    out = _kernel_entry(name, n, fl, by, sec)
    traffic, src = pmc_traffic(name, key, batch, npoints)
    rp, rsrc = committed_profile_avg_us(name, key)
    out.update({'committed_profile_avg_us': rp, 'committed_profile_source': rsrc,
                'traffic': traffic, 'traffic_unit': 'bytes/launch', 'traffic_source': src,
                'selection': 'largest summed in-step time among the launches on the step\'s own stream',
                'timing': 'in-step HIP events, step enqueued behind a spin (no host gaps)'})
    if side:
        sn, sv = sorted(side.items(), key=lambda kv: -kv[1][3])[0]
        out['largest_side_stream_kernel'] = _kernel_entry(sn, *sv)
        out['with_concurrent_side_mfma'] = concurrent_mfma(kp.timeline(), name, int(main))
    gemms = [kv for kv in ranked if any(k in kv[0] for k in ('gemm', 'wgrad', 'fused_bwd'))]
    out['top_kernels'] = [{k: v for k, v in _kernel_entry(nm, *vals).items()
                           if k in ('kernel', 'in_step_ms', 'launches_per_step', 'frac', 'unit', 'compute_unit')}
                          for nm, vals in ranked[:8]]
    mf = [v for k, v in summ.items() if any(t in k for t in ('gemm', 'wgrad', 'fused_bwd', 'knn_wave'))]
    out['executed_gflop_per_step'] = round(sum(v[1] for v in mf) / 1e9, 2)      # MFMA work only
    out['all_engine_gemms_in_step'] = {
        'tflops': round(sum(v[1] for _, v in gemms) / max(sum(v[3] for _, v in gemms), 1e-12) / 1e12, 2),
        'ms_per_step': round(sum(v[3] for _, v in gemms) * 1e3, 3), 'launches': sum(v[0] for _, v in gemms)}
    if replay:      # isolated back-to-back replay of the recorded launches (rewrites outputs: last)
        try:
            rs = kp.replay(name, reps=20)
            out['isolated_replay'] = {'avg_launch_us': round(rs * 1e6, 2), 'tflops': round(fl / n / rs / 1e12, 2)}
        except RuntimeError as e:       # single-launch probes of the non-engine kernels keep no relaunch
            out['isolated_replay'] = f'n/a: {e}'
    return out


def step_roofline(key, npoints, batch, ms, roof=None):
    """Whole-step fraction of the fp32 peak with the reference algorithm's flop count and, when
    the probe ran, with the flops the build executes (the fused EdgeConv / algebraic rewrites
    execute fewer than the reference algorithm: SURVEY.md 8(d))."""
    gf = ALGO_GFLOP_PER_SAMPLE.get((key, npoints))
    if gf is None:
        return None
    tf = gf * batch / (ms * 1e-3) / 1e3
    out = {'algo_gflop_per_sample': gf, 'achieved_tflops_per_gpu': round(tf, 2),
           'frac_of_fp32_peak': round(tf / FP32_PEAK_TFLOPS, 4)}
    if roof and roof.get('executed_gflop_per_step'):
        eg = roof['executed_gflop_per_step'] / batch
        etf = eg * batch / (ms * 1e-3) / 1e3
        out['executed'] = {'gflop_per_sample': round(eg, 3), 'tflops_per_gpu': round(etf, 2),
                           'frac_of_fp32_peak': round(etf / FP32_PEAK_TFLOPS, 4),
                           'source': 'sum of the probed MFMA launches\' algorithmic flops (engine GEMMs, '
                                     'fused backward, kNN distance tiles) in one step'}
    return out


# ----------------------------------------------------------------------------- one workload
def run_workload(key, batch, npoints, args, world, rank, dev):
    import torch
    import torch.distributed as dist
    import pcseg
    from pcseg.ddp import FlatGradAllReduce, broadcast_model
    from pcseg.optim import FlatAdam
    from pcseg.synthetic import make_batch

    name, ctor, kind, _, _, cfg = WORKLOADS[key]
    print(f'[bench] {name}: batch {batch} x {npoints} pts, {args.warmup} warm-up + {args.steps} timed steps',
          file=sys.stderr, flush=True)
    torch.manual_seed(0)
    model = ctor(pcseg).to(dev).train()     # PyTorch default init (random weights)
    pcseg.engine.set_bwd_fuse(model, args.bwd_fuse)
    pcseg.engine.set_edge_inverse(model, args.edge_inverse)
    broadcast_model(model)
    grads = FlatGradAllReduce(model)
    use_graph = args.graph and world == 1
    opt = FlatAdam(grads, lr=1e-3)          # one HIP launch; step count on the device (capturable)
    pts, labels, lengths = make_batch(batch, npoints, seed=1000 * 2 + rank)
    x = model_input(pts.to(dev), kind)
    lab = (labels.float() if kind == 'chfirst6' else labels).to(dev)
    lengths = lengths.to(dev)
    prefetch = hasattr(model, 'prefetch_geometry') and not args.no_prefetch

    in_bwd = args.prefetch_point == 'backward'
    at_start = args.prefetch_point == 'start'

    def step():
        grads.zero_grad()
        if prefetch and in_bwd:
            # pipelined input: the next batch's neighbour search (here the same resident
            # blocks, fresh FPS starts) runs on the side stream under this backward,
            # enqueued from a gradient hook once the first backward stages are queued
            model.prefetch_geometry_in_backward(x)
        if prefetch and at_start:
            model.prefetch_geometry_at_start(x)      # enqueued right after this forward takes its plan
        loss = pcseg.masked_onehot_cross_entropy(logits_of(model(x)), lab, lengths)
        if prefetch and not in_bwd and not at_start:
            model.prefetch_geometry(x)
        loss.backward()
        grads.synchronize()
        opt.step()
        return loss

    eager_step = step
    if use_graph:
        # the whole step in two alternating HIP graphs (pcseg.graphs.CapturedStep): one
        # hipGraphLaunch per step; the next step's geometry still runs under the backward
        from pcseg.graphs import CapturedStep
        cs = CapturedStep(model, x, lab, lengths, grads, opt, pcseg.masked_onehot_cross_entropy, logits_of,
                          warmup=2, prefetch=not args.no_prefetch, geometry=args.graph_geometry)
        prefetch = cs.prefetch

        def step():
            return cs.step()
    prio = contextlib.ExitStack()
    if args.stream_priority == 'high':
        # the step (its critical path) on a high-priority stream; the geometry side stream and the
        # wgrad lane keep normal priority (0), below it, so the hardware queue scheduler hands
        # free CUs to the critical path first
        hs = step_stream(dev)
        hs.wait_stream(torch.cuda.current_stream(dev))
        prio.enter_context(torch.cuda.stream(hs))
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    # PCS_BENCH_STEPLOG=1: per-step host enqueue times, and the main thread's stack whenever one
    # step's enqueue has taken over 200 ms (a host stall: where it blocks)
    steplog = os.environ.get('PCS_BENCH_STEPLOG') == '1'
    th, stalls, cur, mem = [], [], [None], []
    if steplog:
        import threading
        import traceback
        main_id, done = threading.get_ident(), threading.Event()

        def watch():
            while not done.wait(0.1):
                ts = cur[0]
                if ts is not None and time.perf_counter() - ts > 0.2:
                    fr = sys._current_frames().get(main_id)
                    stalls.append(f'+{(time.perf_counter() - ts) * 1e3:.0f} ms: ' +
                                  ' <- '.join(f'{os.path.basename(f.filename)}:{f.lineno}:{f.name}'
                                              for f in reversed(traceback.extract_stack(fr)[-8:])))
        wt = threading.Thread(target=watch, daemon=True)
        wt.start()
    from pcseg import engine as _eng
    w0 = _eng.inflight_wait_s[0] + getattr(opt, 'wait_s', 0.0)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        cur[0] = time.perf_counter()
        loss = step()
        if steplog:
            th.append(time.perf_counter())
            mem.append(torch.cuda.memory_reserved(dev) / 2**30)
    cur[0] = None
    t_host = time.perf_counter() - t0          # host time of the K steps (the step has no host sync)
    # of which waiting on the run-ahead bound (FlatAdam / engine join: max 3 steps ahead)
    t_wait = _eng.inflight_wait_s[0] + getattr(opt, 'wait_s', 0.0) - w0
    if steplog:
        done.set()
        wt.join()
        print(f'[bench] {name} host ms per step: ' + ' '.join(f'{(b - a) * 1e3:.1f}' for a, b in zip([t0] + th, th)),
              file=sys.stderr, flush=True)
        print(f'[bench] {name} reserved GiB per step: ' + ' '.join(f'{m:.0f}' for m in mem), file=sys.stderr, flush=True)
        for x in stalls:
            print(f'[bench] {name} stall {x}', file=sys.stderr, flush=True)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t)
    if not torch.isfinite(loss):
        raise RuntimeError(f'{name}: non-finite loss')
    roof = None
    if not args.no_roofline:
        roof = kernel_roofline(eager_step, dev, key, batch, npoints, replay=args.roofline_replay)
    prio.close()
    torch.cuda.synchronize(dev)
    ms = dt / args.steps * 1e3
    res = {'value': round(world * batch * npoints * args.steps / dt, 1), 'unit': 'points/s',
           'ms_per_step': round(ms, 3),
           'config': {'workload': f'{name} seg, {npoints} pts, batch {batch}/GPU, fwd+CE+bwd'
                                  f'{"+allreduce" if world > 1 else ""}+Adam',
                      'baseline_config': cfg, 'model': name, 'global_batch': world * batch, 'npoints': npoints,
                      'parallelism': f'dp{world}', 'geometry_prefetch': prefetch, 'hip_graph': use_graph,
                      'stream_priority': args.stream_priority},
           'host_enqueue_ms_per_step': round((t_host - t_wait) / args.steps * 1e3, 3),
           'host_runahead_wait_ms_per_step': round(t_wait / args.steps * 1e3, 3),
           'roofline': roof, 'step_roofline': step_roofline(key, npoints, batch, ms, roof)}
    del model, grads, opt
    torch.cuda.empty_cache()
    return res


_STEP_STREAMS: dict = {}


def step_stream(dev):
    """The process's one high-priority step stream per device, reused by every workload: HIP maps
    streams onto its few hardware queues (GPU_MAX_HW_QUEUES = 4) round robin as they are created,
    so a fresh stream per workload eventually shares a queue with pcseg's geometry stream or wgrad
    lane, and the critical path then serialises behind them (round 5: PointNeXt-B measured 16.9 ms
    when timed fourth in one process, 9.2 ms alone)."""
    import torch
    hs = _STEP_STREAMS.get(dev)
    if hs is None:
        hs = _STEP_STREAMS[dev] = torch.cuda.Stream(device=dev, priority=torch.cuda.Stream.priority_range()[1])
    return hs


def release_cached(dev):
    """Between workloads: collect the finished workload's objects, then return the caching
    allocator's free blocks to the device, so the next workload allocates into a fresh pool
    instead of the previous one's fragments."""
    import gc
    import torch
    gc.collect()
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()


def run_drop_in(key, batch, npoints, args, dev):
    """The unchanged harness-A step (Training/training.py:56-60) on the pcseg model: torch.optim.Adam
    over model.parameters(), optimizer.zero_grad() (grads set to None), outputs = model(points),
    loss = criterion(...), loss.backward(), optimizer.step() -- on the default stream, with no
    geometry prefetch and no flat gradient / optimizer buffers.  Also timed with the harness's
    per-step `loss.item()` host sync (training.py:71).  Inputs resident in HBM as in `value`."""
    import torch
    import pcseg
    from pcseg.synthetic import make_batch

    name, ctor, kind, _, _, _ = WORKLOADS[key]
    torch.manual_seed(0)
    model = ctor(pcseg).to(dev).train()
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    pts, labels, lengths = make_batch(batch, npoints, seed=2000)
    x = model_input(pts.to(dev), kind)
    lab = (labels.float() if kind == 'chfirst6' else labels).to(dev)
    lengths = lengths.to(dev)

    def step():
        opt.zero_grad()
        loss = pcseg.masked_onehot_cross_entropy(logits_of(model(x)), lab, lengths)
        loss.backward()
        opt.step()
        return loss

    from pcseg import engine as _eng

    def timed(sync_item):
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize(dev)
        w0 = _eng.inflight_wait_s[0]
        t0 = time.perf_counter()
        for _ in range(args.steps):
            loss = step()
            if sync_item:
                float(loss.item())
        # host time of the steps, less the engine's run-ahead waits (end-of-backward join)
        t_host = time.perf_counter() - t0 - (_eng.inflight_wait_s[0] - w0)
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / args.steps * 1e3, t_host / args.steps * 1e3

    ms, host = timed(False)
    ms_sync, _ = timed(True)
    roof = None if args.no_roofline else kernel_roofline(step, dev, key, batch, npoints)
    out = {'ms_per_step': round(ms, 3), 'value': round(batch * npoints / (ms * 1e-3), 1), 'unit': 'points/s',
           'host_enqueue_ms_per_step': round(host, 3),
           'ms_per_step_with_loss_item_sync': round(ms_sync, 3),
           'step': 'Training/training.py:56-60 unchanged: torch.optim.Adam, zero_grad(set_to_none), forward, '
                   'criterion, backward, step; default stream, no geometry prefetch',
           'roofline': roof, 'step_roofline': step_roofline(key, npoints, batch, ms, roof)}
    del model, opt
    torch.cuda.empty_cache()
    return out


# ----------------------------------------------------------------------------- the JSON line
LINE_LIMIT = 4096       # the driver reads the last ~10 KB of stdout+stderr: the line stays far below


def full_record(results, cpu_res, args, world, rccl_world, keys, others):
    """Everything the run measured (the detail file's content): the primary workload at the top
    level, the second half of the metric under `secondary`, the per-GPU halves of configs[3] /
    configs[4] under `other_configs`."""
    prim = results[args.model]
    res = {'metric': METRIC, 'value': prim['value'], 'unit': 'points/s', 'n_gpus': world,
           'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': prim['ms_per_step'],
           'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': 'fp32',
           'data': 'synthetic S3DIS-like blocks (pcseg.synthetic), random-init weights',
           'config': dict(prim['config'], rccl_world=rccl_world),
           'host_enqueue_ms_per_step': prim['host_enqueue_ms_per_step'],
           'host_runahead_wait_ms_per_step': prim.get('host_runahead_wait_ms_per_step'),
           'roofline': prim['roofline'], 'step_roofline': prim['step_roofline'],
           'drop_in': prim.get('drop_in'), 'cpu_baseline': cpu_res.get(args.model)}
    for k in keys[1:]:
        res['secondary'] = dict(results[k], metric=METRIC, n_gpus=world, dtype='fp32', cpu_baseline=cpu_res.get(k))
    if others:
        res['other_configs'] = {k: dict(results[k], metric=METRIC, n_gpus=world, dtype='fp32', cpu_baseline=None)
                                for k in others}
    return res


def write_detail(full, path):
    """The full record (top kernels, side-stream kernels, concurrent MFMA, drop-in rooflines, the
    all-core CPU leg) as a side file; returns its repo-relative path, or None when not written."""
    if not path or path == 'none':
        return None
    path = path if os.path.isabs(path) else os.path.join(REPO, path)
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, 'w') as f:
            json.dump(full, f, indent=1)
    except OSError as e:
        print(f'[bench] detail file not written: {e}', file=sys.stderr, flush=True)
        return None
    return os.path.relpath(path, REPO)


def _r(x, nd=4):
    return None if x is None else round(x, nd)


def compact_roofline(roof):
    """The dominant kernel's roofline, the contract's fields only."""
    if not roof:
        return None
    out = {'kernel': roof['kernel'].replace('pcs::', ''), 'bound': roof['bound'], 'achieved': roof['achieved'],
           'peak': roof['peak'], 'unit': roof['unit'], 'frac': roof['frac'], 'traffic': roof.get('traffic'),
           'avg_launch_us': roof['avg_launch_us'], 'launches_per_step': roof['launches_per_step']}
    by = roof.get('algo_bytes_per_launch')
    if out['traffic'] and by:
        out['traffic_over_algo'] = round(out['traffic'] / by, 3)
    if roof.get('committed_profile_avg_us') is not None:
        out['committed_profile_avg_us'] = roof['committed_profile_avg_us']
    return out


def compact_cpu(cb):
    if not cb:
        return None
    return {'value': _r(cb.get('value'), 1), 'unit': cb.get('unit', 'points/s'), 'cores': cb.get('cores'),
            'kind': cb.get('kind', 'port'), 'sample': (cb.get('sample') or '')[:200]}


def compact_workload(r, with_cpu=True):
    out = {'value': r['value'], 'unit': 'points/s', 'ms_per_step': r['ms_per_step'],
           'workload': r['config']['workload'], 'roofline': compact_roofline(r.get('roofline'))}
    sr = r.get('step_roofline')
    if sr:
        out['step_frac_fp32'] = sr['frac_of_fp32_peak']
    if with_cpu:
        out['cpu_baseline'] = compact_cpu(r.get('cpu_baseline'))
    di = r.get('drop_in')
    if di:
        out['drop_in'] = {'ms_per_step': di['ms_per_step'], 'host_enqueue_ms': di['host_enqueue_ms_per_step']}
    return out


def compact_line(full, detail_path):
    """The one JSON line bench.py prints last: the contract's keys, the compact roofline and CPU
    baseline of both halves of the metric, a summary per other config, and the detail file's
    path.  Kept under LINE_LIMIT bytes (the long strings are trimmed first if it is not)."""
    line = {k: full[k] for k in ('metric', 'value', 'unit', 'n_gpus', 'steps', 'warmup', 'ms_per_step',
                                 'higher_is_better', 'scaling', 'vs_baseline', 'dtype', 'data')}
    c = full['config']
    line['config'] = {k: c[k] for k in ('workload', 'model', 'global_batch', 'npoints', 'parallelism',
                                        'rccl_world') if k in c}
    line['roofline'] = compact_roofline(full.get('roofline'))
    line['cpu_baseline'] = compact_cpu(full.get('cpu_baseline'))
    sr = full.get('step_roofline')
    line['step_frac_fp32'] = sr['frac_of_fp32_peak'] if sr else None
    di = full.get('drop_in')
    if di:
        line['drop_in'] = {'ms_per_step': di['ms_per_step'], 'host_enqueue_ms': di['host_enqueue_ms_per_step']}
    line['host_enqueue_ms_per_step'] = full.get('host_enqueue_ms_per_step')
    if full.get('secondary'):
        line['secondary'] = compact_workload(full['secondary'])
    if full.get('other_configs'):
        line['other_configs'] = {
            k: {'value': r['value'], 'ms_per_step': r['ms_per_step'],
                'frac': (r.get('roofline') or {}).get('frac'),
                'drop_in_ms': (r.get('drop_in') or {}).get('ms_per_step')}
            for k, r in full['other_configs'].items()}
    line['detail'] = detail_path
    if len(json.dumps(line, separators=(',', ':'))) > LINE_LIMIT:
        for blk in (line, line.get('secondary') or {}):
            if blk.get('cpu_baseline'):
                blk['cpu_baseline']['sample'] = blk['cpu_baseline']['sample'][:60]
        line['data'] = 'synthetic'
    if len(json.dumps(line, separators=(',', ':'))) > LINE_LIMIT:
        line.pop('other_configs', None)
    return line


def emit_line(full, detail_out):
    """Write the detail file, then print the compact line as the LAST line of stdout (stderr is
    flushed first, so no progress line lands after it in a merged log)."""
    detail = write_detail(full, detail_out)
    line = json.dumps(compact_line(full, detail), separators=(',', ':'))
    sys.stderr.flush()
    print(line, flush=True)
    return line


# ----------------------------------------------------------------------------- launcher
def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def spawn_ranks(n):
    """Start n rank processes of this script (torchrun-style env), before this process has
    touched the GPU; exit with the worst return code."""
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR='127.0.0.1', MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    return max(rcs, key=abs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=30)
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--model', default='pointnetpp', choices=sorted(WORKLOADS))
    ap.add_argument('--secondary', default='auto', help="second workload on the same line ('auto': dgcnn when "
                                                        "--model is pointnetpp; 'none' to skip)")
    ap.add_argument('--others', default='auto',
                    help="further workloads timed on the same line under `other_configs`, comma-separated "
                         "('auto': BASELINE configs[3] / configs[4]'s per-GPU halves -- pointnetpp_msg at batch 32, "
                         "pointnext at batch 16 x 24576 -- when --model is pointnetpp; 'none' to skip); no CPU "
                         "baseline for them")
    ap.add_argument('--batch', type=int, default=0, help='per-GPU batch (default: the workload\'s)')
    ap.add_argument('--npoints', type=int, default=0, help='points per block (default: the workload\'s)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-batch', type=int, default=0, help='CPU baseline batch (default: the GPU batch)')
    ap.add_argument('--cpu-steps', type=int, default=5)
    ap.add_argument('--cpu-budget', type=float, default=40.0, help='seconds of timed CPU steps per workload')
    ap.add_argument('--cpu-threads', type=int, default=0)
    ap.add_argument('--cpu-baseline-worker', action='store_true')
    ap.add_argument('--no-roofline', action='store_true')
    ap.add_argument('--no-drop-in', action='store_true',
                    help='skip the unchanged harness-A step (torch.optim.Adam, default stream, no prefetch) '
                         'reported as `drop_in` beside each workload (N=1 only)')
    ap.add_argument('--roofline-replay', action='store_true',
                    help='also time the dominant kernel\'s launches replayed back to back (rewrites outputs)')
    ap.add_argument('--graph', action='store_true',
                    help='capture the training step in HIP graphs (pcseg.graphs.CapturedStep) and time its replays '
                         '(N=1 only; multi-GPU steps run eagerly)')
    ap.add_argument('--prefetch-point', choices=['backward', 'loss', 'start'], default='loss',
                    help="where the next step's geometry is enqueued: between the loss and backward() (default) "
                         "or from a gradient hook inside the backward (round 2 A/B: within noise, 5.50 vs 5.52 ms)")
    ap.add_argument('--no-prefetch', action='store_true',
                    help='do not enqueue the next step\'s FPS/ball-query/3-NN before this step\'s backward')
    ap.add_argument('--graph-geometry', choices=['graph', 'eager'], default='graph',
                    help="--graph: capture the next step's neighbour search too, or enqueue it eagerly per step")
    ap.add_argument('--stream-priority', choices=['default', 'high'], default='high',
                    help='run the step on a high-priority stream (default; pcseg\'s side streams -- the next '
                         'step\'s geometry, the wgrad lane -- keep normal priority, below it) or on the default stream')
    ap.add_argument('--edge-inverse', choices=['side', 'backward', 'deferred'], default='deferred',
                    help='DGCNN: where the EdgeConv backward\'s inverse kNN maps are built: on the side stream '
                         'after the last EdgeConv (deferred, default), right after each EdgeConv (side), or in '
                         'the backward')
    ap.add_argument('--bwd-fuse', choices=['default', 'off', 'all'], default='default',
                    help='backward kernel choice of the shared-MLP stacks (pcs_mlp_layer.bwd_fuse; A/B runs)')
    ap.add_argument('--detail-out', default='gpurun_out/bench_detail.json',
                    help="where the full record (top kernels, side streams, drop-in rooflines, ...) is written; "
                         "the printed line names it ('none': not written)")
    ap.add_argument('--check-launch', action='store_true',
                    help='launcher self-test: each rank joins a gloo group, prints its env as JSON, exits (no GPU)')
    args = ap.parse_args()
    if args.cpu_baseline_worker:
        cpu_baseline_worker(args)
        return 0
    if args.gpus < 1:
        raise SystemExit('--gpus must be >= 1')
    if 'WORLD_SIZE' not in os.environ and args.gpus > 1:
        return spawn_ranks(args.gpus)
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus:
        raise SystemExit(f'bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks')

    import torch.distributed as dist
    if args.check_launch:
        dist.init_process_group('gloo', rank=rank, world_size=world)
        print(json.dumps({'rank': rank, 'local_rank': local, 'world': dist.get_world_size(),
                          'master': f"{os.environ.get('MASTER_ADDR')}:{os.environ.get('MASTER_PORT')}"}),
              flush=True)
        dist.barrier()
        dist.destroy_process_group()
        return 0

    keys = [args.model]
    sec = args.secondary
    if sec == 'auto':
        sec = 'dgcnn' if args.model == 'pointnetpp' else 'none'
    if sec != 'none':
        if sec not in WORKLOADS:
            raise SystemExit(f'unknown --secondary {sec}')
        keys.append(sec)
    oth = args.others
    if oth == 'auto':
        oth = 'pointnetpp_msg,pointnext' if args.model == 'pointnetpp' else 'none'
    others = [] if oth == 'none' else [k for k in oth.split(',') if k and k not in keys]
    for k in others:
        if k not in WORKLOADS:
            raise SystemExit(f'unknown --others workload {k}')
    sizes = {k: (args.batch or WORKLOADS[k][3], args.npoints or WORKLOADS[k][4]) if k == args.model
             else (WORKLOADS[k][3], WORKLOADS[k][4]) for k in keys + others}

    cpu_res = {}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        for k in keys:                          # before the GPU run: the host is otherwise idle
            cpu_res[k] = run_cpu_baseline(args, k, *sizes[k])

    import torch
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f'RCCL world {dist.get_world_size()} != --gpus {args.gpus}')
    dev = torch.device('cuda', local)

    results = {}
    for k in keys + others:
        results[k] = run_workload(k, *sizes[k], args, world, rank, dev)
        release_cached(dev)     # the model, its closures and plans are gone: hand their blocks back
    if world == 1 and not args.no_drop_in:
        for k in keys + others:
            print(f'[bench] {k}: drop-in harness-A step', file=sys.stderr, flush=True)
            results[k]['drop_in'] = run_drop_in(k, *sizes[k], args, dev)
            release_cached(dev)
    if rank == 0:
        full = full_record(results, cpu_res, args, world,
                           dist.get_world_size() if world > 1 else 1, keys, others)
        emit_line(full, args.detail_out)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == '__main__':
    sys.exit(main())
