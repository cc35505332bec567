#!/usr/bin/env python3
"""bench.py -- SRF training-step throughput (acoustic frames/sec) on MI355X.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Headline workload (the metric's "3-iter DR at 1/2/4/8 MI355X" = BASELINE.json
configs[3], C4, whose per-GPU batch fits one GPU): WSJ SRF L=6, PH=CH=16, DIM=32,
LPAD=RPAD=2, DR iter 3, fp32, class_n 32; per GPU B=28 utterances of T=800 frames
(the reference's bucket rule for 24000 frames/batch).  The TIMIT C2
model (configs[1]: L=3, PH=CH=8, DIM=16, LPAD=RPAD=4, B=17, T=320) is measured
after it and reported under "extra".  Synthetic N(0,1) 123-d fbank, labels
uniform in [1, C-2], L = T'/2.
One step = process_train_step: crop, forward, CTC, backward, RCCL gradient
all-reduce (N > 1), fused Adam.  value = sum(inp_len) over all ranks / step time
(the reference's frame counter, trainer_sr.py:74), weak scaling.

Prints ONE JSON line on rank 0 (roofline of the dominant kernel from HIP events
inside the timed region; CPU baseline = torch-CPU op-for-op mirror of
sequence_router_naive.py on a bounded sample, rank 0 at N=1 only, on all host
threads and on one core).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

WORKLOADS = {
    # name: (config kwargs, class_n, per-GPU B, T)
    'timit_c2': (dict(enc=3, iters=3, lpad=4, rpad=4, ph=8, pd=16, ch=8, cd=16, vd=16, context=False), 63, 17, 320),
    'wsj_c4': (dict(enc=6, iters=3, lpad=2, rpad=2, ph=16, pd=32, ch=16, cd=32, vd=32, context=False), 32, 28, 800),
    'wsj_c3': (dict(enc=6, iters=3, lpad=2, rpad=2, ph=16, pd=32, ch=16, cd=32, vd=32, context=True), 32, 28, 800),
    # BASELINE C5 (HBM-bound stress): PH=CH=16 assumed as in C3; fp32 pose
    # (the parity path) and, as BASELINE names it, the opt-in fp8 (e4m3) pose MFMA
    'wsj_c5': (dict(enc=8, iters=5, lpad=20, rpad=20, ph=16, pd=64, ch=16, cd=64, vd=64, context=True), 32, 28, 800),
    'wsj_c5_fp8': (dict(enc=8, iters=5, lpad=20, rpad=20, ph=16, pd=64, ch=16, cd=64, vd=64, context=True,
                        pose_fp8=True), 32, 28, 800),
}
FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix (= vector) peak
BF16_MFMA_PEAK_TFLOPS = 2500.0  # dense bf16 / f16 MFMA peak
HBM_PEAK_GBS = 8000.0
# rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of `bench.py`, averaged per dispatch by
# scripts/pmcsum.py (KiB per dispatch), per workload
PMC_TRAFFIC = {'timit_c2': os.path.join(HERE, 'profiles', 'r05_pmc_traffic_c2.json'),
               'wsj_c4': os.path.join(HERE, 'profiles', 'r06_pmc_c4.json')}


def make_config(kw):
    from srf_amd.common_helper import build_parser
    ns = build_parser().parse_args([])
    ns.feat_dim = 123
    ns.model_encoder_num = kw['enc']
    ns.model_caps_iter = kw['iters']
    ns.model_caps_window_lpad, ns.model_caps_window_rpad = kw['lpad'], kw['rpad']
    ns.model_caps_primary_num, ns.model_caps_primary_dim = kw['ph'], kw['pd']
    ns.model_caps_convolution_num, ns.model_caps_convolution_dim = kw['ch'], kw['cd']
    ns.model_caps_class_dim = kw['vd']
    ns.model_caps_context = kw['context']
    ns.model_caps_type = 'naive'
    ns.model_pose_fp8 = kw.get('pose_fp8', False)
    ns.model_initializer = 'fan_avg'
    ns.train_lr_param_k, ns.train_warmup_n = 0.5, 1200      # train_srf_timit.sh:49-51
    return ns


def synthetic_batch(B, T, class_n, rank, dev):
    g = torch.Generator().manual_seed(1234 + rank)
    feats = torch.randn(B, T, 123, generator=g)
    Tp = (T + 3) // 4
    L = Tp // 2
    gl = torch.Generator().manual_seed(4321 + rank)
    labels = torch.randint(1, class_n - 1, (B, L), generator=gl, dtype=torch.int32)
    inp_len = torch.full((B,), T, dtype=torch.int32)
    tar_len = torch.full((B,), L, dtype=torch.int32)
    # lengths stay host-side, as the input pipeline yields them (crop without a device sync)
    if str(dev) != 'cpu':
        inp_len = inp_len.pin_memory()
    return feats.to(dev), labels.to(dev), inp_len, tar_len.to(dev)


class HipEvents:
    """Raw hipEvent_t handles from the HIP runtime torch already loaded."""

    def __init__(self):
        self.hip = ctypes.CDLL('libamdhip64.so.7')
        self.hip.hipEventCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        self.hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
        self.hip.hipEventSynchronize.argtypes = [ctypes.c_void_p]

    def create(self, n):
        arr = (ctypes.c_void_p * n)()
        for i in range(n):
            h = ctypes.c_void_p()
            assert self.hip.hipEventCreate(ctypes.byref(h)) == 0
            arr[i] = h.value
        return arr

    def elapsed_ms(self, a, b):
        self.hip.hipEventSynchronize(ctypes.c_void_p(b))
        ms = ctypes.c_float()
        assert self.hip.hipEventElapsedTime(ctypes.byref(ms), ctypes.c_void_p(a), ctypes.c_void_p(b)) == 0
        return ms.value


def _cpu_model():
    try:
        with open('/proc/cpuinfo') as fh:
            for ln in fh:
                if ln.startswith('model name'):
                    return ln.split(':', 1)[1].strip()
    except OSError:
        pass
    return 'unknown'


def usable_cpus():
    """The cores this process may run on: its affinity mask, bounded by the cgroup CPU
    quota when one is set (a container whose affinity lists every core of the machine
    but whose quota grants 16 runs 16 threads at a time; more threads only contend)."""
    n = len(os.sched_getaffinity(0))
    try:
        with open('/sys/fs/cgroup/cpu.max') as fh:
            quota, period = fh.read().split()[:2]
        if quota != 'max':
            n = min(n, max(1, -(-int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def cpu_baseline(model_gpu, cfg, class_n, T, seconds, threads=None, max_steps=50):
    """torch-CPU op-for-op mirror of naive (oracle/naive_mirror.py), fp32,
    one T-frame utterance per step, timed for >= `seconds` (>= 1 step)."""
    from oracle import naive_mirror as nm
    from oracle import srf_oracle as so
    kw = dict(feat_dim=123, enc_num=cfg.model_encoder_num, iters=cfg.model_caps_iter,
              lpad=cfg.model_caps_window_lpad, rpad=cfg.model_caps_window_rpad, ph=cfg.model_caps_primary_num,
              pd=cfg.model_caps_primary_dim, ch=cfg.model_caps_convolution_num, cd=cfg.model_caps_convolution_dim,
              vd=cfg.model_caps_class_dim, class_n=class_n, context=bool(cfg.model_caps_context))
    shape = so.SrfShape(**kw)
    if threads is None:
        threads = usable_cpus()   # every core this process may run on
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    params = model_gpu.export_params()
    mirror = nm.NaiveMirror(shape, params, dtype=torch.float32)
    opt = nm.TfAdam(mirror.parameters(), k=0.5, warmup=1200)
    feats, labels, inp_len, tar_len = synthetic_batch(1, T, class_n, 0, 'cpu')
    frames, steps = 0, 0
    t0 = time.perf_counter()
    while True:
        nm.train_step(mirror, opt, feats, labels, inp_len, tar_len)
        frames += int(inp_len.sum())
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds or steps >= max_steps:
            break
    torch.set_num_threads(prev)
    return {'value': round(frames / el, 1), 'unit': 'frames/s', 'cores': threads, 'kind': 'port',
            'cpu_model': _cpu_model(),
            'sample': f'{steps} train steps x 1 utterance x {T} frames (torch-CPU mirror of '
                      f'sequence_router_naive.py, fp32, {el:.1f}s)'}


def pmc_traffic(path, kernels, weights):
    """HBM bytes per launch of the timed routing passes, from the committed PMC passes:
    2 x FETCH_SIZE + WRITE_SIZE (gfx950 tallies wide streaming reads at half their bytes,
    MI355X_MICROARCH.md HBM section), for the largest-grid dispatch of each kernel (the
    last layer), averaged with the pass weights.  None when no profile is committed."""
    try:
        with open(path) as fh:
            rows = json.load(fh)
    except (OSError, ValueError):
        return None
    total = 0.0
    for name, w in zip(kernels, weights):
        bare = name.replace('void ', '')
        cand = [r for r in rows if r['kernel'].replace('void ', '').startswith(bare)
                and 'FETCH_SIZE' in r and 'WRITE_SIZE' in r]
        if not cand:
            return None
        r = max(cand, key=lambda r: r['grid'])
        total += w * (2.0 * r['FETCH_SIZE'] + r['WRITE_SIZE']) * 1024.0
    return total / sum(weights)


def _timed(step, steps, world, dev):
    """Barrier + synchronize on both sides of `steps` calls; max over ranks."""
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def sdr_roofline(model, tms, group=1):
    """HBM roofline of the SDR recurrence (the last layer's forward launches, one
    workgroup per utterance walking its frames; sequence_router_naive.py:162-170).
    Algorithmic bytes per frame: the frame's u_t read once per routing iteration by
    the streaming kernel (route_sdr_stream.hip, frames beyond the register budget) or
    once in all by the register-resident one (route_sdr_seq.hip), plus v_t written."""
    from srf_amd import _lib
    in_n, J, D, Din = model.layer_shapes[model.enc_num - 1]
    R = model.route_iters
    stream = bool(_lib.lib().srf_route_sdr_couplings_required(in_n, J, D, R))
    reads = R if stream else 1
    elt = 2 if (stream and model.pose_fp8 and model.sdr_options.get('u_bf16', True)) else 4   # bf16 u
    per_frame = reads * in_n * J * D * elt + J * D * 4
    ms = sum(t for t, _ in tms)
    frames = sum(f for _, f in tms)
    if not tms or ms <= 0:
        return None
    gbs = per_frame * frames / (ms * 1e-3) / 1e9
    return {'kernel': ('sdr_stream_fwd_kernel<%d,%d>' % (D, J * D // 64) if stream else
                       'sdr_seq_fwd_kernel<%d,%d,...>' % (D, J)) +
            ' (layer %d SDR recurrence, forward, %s per utterance)' % (
                model.enc_num, 'one workgroup' if group <= 1 else '%d workgroups' % group),
            'bound': 'hbm', 'achieved': round(gbs, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'frac': round(gbs / HBM_PEAK_GBS, 4), 'traffic': None,
            'avg_launch_us': round(ms / len(tms) * 1e3, 2), 'bytes_per_launch': per_frame * frames / len(tms),
            'bytes_per_frame': per_frame, 'note': 'u_t (%s) read %d time(s) per frame' % ('bf16' if elt == 2 else 'fp32',
                                                                                     reads)}


def measure(workload, args, world, rank, dev, flag_group=None):
    """One workload: W eager + W graphed warmup steps, K timed training steps (the
    hipGraph replay of forward + CTC + backward, then the all-reduce and Adam), K
    eager steps with HIP events around the last layer's forward routing passes,
    and K forward-only passes."""
    from srf_amd import train_helper, trainer_sr
    from srf_amd.sequence_router import SequenceRouter

    kw, class_n, B, T = WORKLOADS[workload]
    cfg = make_config(kw)
    model = SequenceRouter(cfg, None, class_n, device=dev, seed=1234)   # same init on every rank
    if args.sdr_separate_gxgw:
        from srf_amd import ops
        ops.SDR_FUSED_GXGW = False
    if args.sdr_capsnorm_per_layer:
        from srf_amd import ops
        ops.SDR_CAPSNORM_BATCHED = False
    if args.sdr_gu_factors:
        from srf_amd import ops
        ops.SDR_GU_FACTORS = True
    if args.sdr_last_gxw_inline:
        from srf_amd import ops
        ops.SDR_LAST_GXW_SIDE = False
    if args.side_streams:
        from srf_amd import ops
        ops.DR_GW_SIDE = ops.CNNFE_WGRAD_SIDE = True
    if args.dr_chunks:
        # "l:c,l:c" input-capsule chunks of DR layer l's routing passes (A/B of the plan's choice)
        for item in args.dr_chunks.split(','):
            l, c = item.split(':')
            model.n_chunks_override[int(l)] = int(c)
    if args.sdr_last_group is not None:
        g = [int(x) for x in args.sdr_last_group.split(',')]
        model.sdr_options['last_group'] = (g[0], g[-1])
    # N > 1: the gradient all-reduce in 25 MB buckets launched as the backward completes
    # them, captured inside the step's hipGraph with the backward they overlap
    # (trainer_sr.GradBuckets; --flat-allreduce: one all-reduce after each replay)
    bucketed = world > 1 and not args.flat_allreduce
    if bucketed:
        trainer_sr.use_grad_buckets(model, 25.0)
    opt = train_helper.get_optimizer(cfg)
    batch = synthetic_batch(B, T, class_n, rank, dev)
    loss_state, frame_state, samples = trainer_sr.Mean(), trainer_sr.Mean(), trainer_sr.Sum()

    def eager_step():
        trainer_sr.process_train_step(4, batch, model, opt, loss_state, frame_state, world, class_n - 1, samples)

    for _ in range(args.warmup):
        eager_step()
    torch.cuda.synchronize()
    graphed = None
    if args.eager:
        step = eager_step
    else:
        # forward + CTC + backward as one hipGraph; all-reduce and Adam eager per step.
        # With buckets the capture holds their collectives: if any rank fails it, every
        # rank falls back to the flat all-reduce (agreed over a gloo group)
        def capture():
            return trainer_sr.GraphedTrainStep(4, batch, model, opt, world, class_n - 1)

        def flat():
            trainer_sr.use_grad_buckets(model, None)
            return capture()
        if bucketed:
            graphed, err = trainer_sr.capture_agreed(capture, flat, flag_group)
            if err is not None:
                bucketed = False
                print(f'[bench] capturing the bucketed all-reduce failed ({err}); flat all-reduce on every rank',
                      file=sys.stderr)
        else:
            graphed = capture()
        for _ in range(args.warmup):
            graphed(loss_state, frame_state, samples)
        torch.cuda.synchronize()

        def step():
            graphed(loss_state, frame_state, samples)

    # HIP events around the dominant kernel (forward routing passes of the last
    # layer), recorded on the launch stream
    ev = HipEvents()
    Tp = (T + 3) // 4
    last = model.enc_num - 1
    geom = model._geom(last, B, Tp)
    R = model.iter
    dr = not model.is_context    # the event hook times DR passes; SDR runs no such pass
    ev_pairs = [(ev.create(R), ev.create(R)) for _ in range(args.steps)] if dr else []
    if dr and args.eager:
        geom.timing = [(ctypes.cast(a, ctypes.c_void_p), ctypes.cast(b, ctypes.c_void_p), R) for a, b in ev_pairs]

    elapsed = _timed(step, args.steps, world, dev)
    geom.timing = None
    if dr and not args.eager:
        # graph replays carry no per-kernel events: time the same kernels in as many
        # eager steps right after the timed region (same shapes, same stream)
        geom.timing = [(ctypes.cast(a, ctypes.c_void_p), ctypes.cast(b, ctypes.c_void_p), R) for a, b in ev_pairs]
        for _ in range(args.steps):
            eager_step()
        torch.cuda.synchronize()
        geom.timing = None
    if graphed is not None:
        graphed.close()

    # forward-only frames/s: model(feats, training=False) as in
    # process_valid_step (BN moving statistics, no dropout), eager launches, outside
    # the training-step timed region, same barrier + max-over-ranks timing
    feats_b, il_b = batch[0], batch[2]
    with torch.no_grad():
        for _ in range(max(1, args.warmup)):
            model(feats_b, input_lengths=il_b, training=False)
        fwd_elapsed = _timed(lambda: model(feats_b, input_lengths=il_b, training=False), args.steps, world, dev)

    sdr_roof = None
    if not dr:
        # SDR: HIP events (on the launch stream) around the last layer's forward
        # recurrence launches of eager forward passes, after the timed region
        plan = model._stack_plan(B, Tp)
        plan.timing = []
        with torch.no_grad():
            for _ in range(max(1, min(args.steps, 3))):
                model(feats_b, input_lengths=il_b, training=False)
        torch.cuda.synchronize()
        tms = [(e0.elapsed_time(e1), fr) for e0, e1, fr in plan.timing]
        plan.timing = None
        sdr_roof = sdr_roofline(model, tms, plan.group(plan.L - 1, dev))

    kern_ms = [ev.elapsed_ms(a[r], b[r]) for a, b in ev_pairs for r in range(R)]
    kern_avg_ms = sum(kern_ms) / len(kern_ms) if kern_ms else float('nan')
    in_n, J, D, Din = model.layer_shapes[last]
    fwd32 = Din in (8, 16, 32) and D in (8, 16, 32) and Din <= D and J * D <= 1024
    frames_prime = B * Tp
    # algorithmic FLOPs per launch: the layer's pose contraction (once per
    # forward, spread over its R pass launches) + one routing iteration
    pose = 2.0 * in_n * J * D * Din
    route = 4.0 * in_n * J * D
    flops_launch = frames_prime * (pose / R + route)
    achieved_tflops = flops_launch / (kern_avg_ms * 1e-3) / 1e12

    traffic, traffic_src = None, PMC_TRAFFIC.get(workload)
    tw = 4 if (Din < 32 or J * D > 512) else 2     # row tiles per wave (route_fwd32.hip Fwd32Plan::TW)
    # iteration 0: the full-K pass with its finish fused for din = dout = 32, else the chunked GEMM
    first = 'route_fwd32_first_full_kernel' if (Din == 32 and D == 32) else f'void route_fwd32_first_kernel<{Din}, {D}>'
    # r >= 1: the software-pipelined pass where it has two row tiles per wave (route_fwd32.hip launch_rpass)
    rpass = f'void route_fwd32{"p" if tw <= 2 else ""}_kernel<{Din}, {D}, 8, {tw}>'
    if fwd32 and traffic_src:
        traffic = pmc_traffic(traffic_src, [first, rpass], [1.0, R - 1.0])
    res = {
        'value': round(B * T * world * args.steps / elapsed, 1), 'ms_per_step': round(elapsed / args.steps * 1e3, 4),
        'config': {'workload': f'{workload}: SRF L={cfg.model_encoder_num} PH=CH={cfg.model_caps_primary_num} '
                               f'DIM={cfg.model_caps_primary_dim} LPAD=RPAD={cfg.model_caps_window_lpad} '
                               f'{"SDR" if model.is_context else "DR"} iter={cfg.model_caps_iter}, '
                               f'{"fp8 (e4m3) pose MFMA, " if model.pose_fp8 else ""}'
                               f'train step (fwd+bwd+allreduce+Adam)',
                   'utterances_per_gpu': B, 'frames_per_utterance': T, 'global_batch': B * world,
                   'parallelism': f'dp{world}',
                   'allreduce': (None if world == 1 else
                                 'RCCL SUM in 25 MB buckets launched as the backward completes them, captured in '
                                 'the step graph' if bucketed else 'one flat RCCL SUM after each replay'),
                   'launch': 'eager' if args.eager else 'hipgraph (fwd+CTC+bwd)'},
        'roofline': {'kernel': (f'{first.replace("void ", "")} + {rpass.replace("void ", "")} (layer {last + 1} DR '
                                f'forward passes, R={R}; pose on v_mfma_f32_32x32x16_f16 as 2-term fp16 splits of '
                                f'power-of-two scaled operands + one bf16 bias MFMA = fp32-accurate)'
                                if fwd32 else f'route_pass_kernel<{Din},{D},8,FWD> (layer {last + 1} DR forward pass)'),
                     'bound': 'mfma', 'achieved': round(achieved_tflops, 3), 'peak': FP32_MFMA_PEAK_TFLOPS,
                     'unit': 'TFLOP/s', 'frac': round(achieved_tflops / FP32_MFMA_PEAK_TFLOPS, 4),
                     'traffic': round(traffic) if traffic else None,
                     'traffic_source': (os.path.relpath(traffic_src, HERE) + ' (HBM bytes per launch, '
                                        '2*FETCH_SIZE+WRITE_SIZE)') if traffic else None,
                     'avg_launch_us': round(kern_avg_ms * 1e3, 2),
                     'flops_per_launch': flops_launch,
                     # what the matrix cores execute: the full pose every pass, per 32-row tile and
                     # capsule 3 f16 K=16 products + 1 bf16 bias product (din 16), 2 + 1 (din 8,
                     # two planes packed in K) or 6 + 1 (din 32, two K=16 halves), on the
                     # 32x32-padded rows
                     'executed_mfma': ({'dtype': 'f16/bf16', 'peak_tflops': BF16_MFMA_PEAK_TFLOPS,
                                        'frac': round(frames_prime * 2.0 * in_n * ((J * D + 31) // 32 * 32) * 16
                                                      * {8: 3, 16: 4, 32: 7}[Din] / (kern_avg_ms * 1e-3) / 1e12
                                                      / BF16_MFMA_PEAK_TFLOPS, 4)} if fwd32 else None)}
                    if dr else sdr_roof,
        'dtype': 'fp8 pose (e4m3, fp32 accumulate) / fp32' if model.pose_fp8 else 'fp32',
        'forward_only': {'value': round(B * T * world * args.steps / fwd_elapsed, 1), 'unit': 'frames/s',
                         'ms_per_step': round(fwd_elapsed / args.steps * 1e3, 4),
                         'mode': 'model(feats, training=False), eager launches'},
    }
    from srf_amd import ops
    ops.check_faults()   # a grouped SDR recurrence that timed out made this run's results wrong
    return res, model, cfg, class_n, T


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--workload', default='wsj_c4', choices=sorted(WORKLOADS),
                    help='the headline line (BASELINE metric: 3-iter DR on the WSJ C4 model)')
    ap.add_argument('--extra', default='timit_c2',
                    help='comma-separated workloads also measured, reported under "extra" (empty: none)')
    ap.add_argument('--cpu-seconds', type=float, default=15.0)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--sdr-last-group', default=None,
                    help='SDR stack: workgroups per utterance of the last layer\'s recurrence, "G" or '
                         '"G_forward,G_backward" (default: SdrStackPlan.group)')
    ap.add_argument('--sdr-separate-gxgw', action='store_true',
                    help='SDR stack: the gx and gW launches of din-32 layers separately (default: fused)')
    ap.add_argument('--sdr-gu-factors', action='store_true',
                    help='SDR stack: the recurrence backward writes gu factors and gx / gW form gu from them '
                         '(default: gu; A/B)')
    ap.add_argument('--sdr-capsnorm-per-layer', action='store_true',
                    help='SDR stack: one LN/dropout launch per inner layer and range (default: one per diagonal)')
    ap.add_argument('--side-streams', action='store_true',
                    help='DR gW / gbias and the CNN-FE stage-2 weight gradient on a side stream (A/B only: '
                         'replays of a captured step then give wrong W / b gradients at times, ops.DR_GW_SIDE)')
    ap.add_argument('--dr-chunks', default='',
                    help='DR: input-capsule chunks per layer, "l:c,..." (default: the plan\'s choice; A/B)')
    ap.add_argument('--sdr-last-gxw-inline', action='store_true',
                    help='SDR stack: the last layer\'s gx / gW on its recurrence\'s stream (default: a side stream)')
    ap.add_argument('--flat-allreduce', action='store_true',
                    help='N > 1: one flat all-reduce after each step instead of backward-overlapped buckets (A/B)')
    ap.add_argument('--eager', action='store_true', help='launch every kernel from Python each step (no hipGraph)')
    args = ap.parse_args()

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    # SRF_DIST_BACKEND=gloo rehearses the multi-rank path on one GPU (ranks share it)
    backend = os.environ.get('SRF_DIST_BACKEND', 'nccl')
    if backend != 'nccl':
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    if world > 1:
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)
        else:
            dist.init_process_group(backend)

    # a CPU side group for host-side agreements (the capture fallback), made on every rank
    flag_group = None
    if world > 1:
        flag_group = dist.group.WORLD if backend == 'gloo' else dist.new_group(backend='gloo')
    res, model, cfg, class_n, T = measure(args.workload, args, world, rank, dev, flag_group)
    line = {
        'metric': 'acoustic frames/sec through SRF (123-d fbank, 3-iter DR) at 1/2/4/8 MI355X',
        'value': res['value'], 'unit': 'frames/s', 'n_gpus': world, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': res['ms_per_step'], 'higher_is_better': True,
        'scaling': 'weak', 'vs_baseline': None, 'dtype': res['dtype'],
        'data': 'synthetic (N(0,1) 123-d fbank, random init)',
        'config': res['config'], 'roofline': res['roofline'], 'forward_only': res['forward_only'],
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the full host (every usable core: affinity mask within the cgroup quota) on one utterance of the workload's
        # length, and one core on a quarter-length utterance (frames/s is per frame)
        cb = cpu_baseline(model, cfg, class_n, T, args.cpu_seconds)
        one = cpu_baseline(model, cfg, class_n, max(40, T // 4), args.cpu_seconds / 2, threads=1)
        cb['one_core'] = {k: one[k] for k in ('value', 'cores', 'sample')}
        line['cpu_baseline'] = cb
    del model
    extra = [w for w in args.extra.split(',') if w and w != args.workload]
    if extra:
        line['extra'] = {}
        for w in extra:
            r, m, _, _, _ = measure(w, args, world, rank, dev, flag_group)
            del m
            line['extra'][w] = r
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
