#!/usr/bin/env python3
"""Benchmark of the BPE merge-training hot path (findNextMerge + applyMerge, core.ts:247-360) on
MI355X.  One step = one merge iteration: a full pair-count pass over the corpus resident in HBM,
the argmax with the reference's tie-break, and the in-place rewrite.

Workload (BASELINE.json configs[2], the single-GPU config the metric is quoted on): a 1 GiB
synthetic latin1 corpus (xorshift32 seed 12345, 256-char alphabet, 1 MiB samples; SURVEY.md
§8(d)) per GPU, mergeUntil({min_weight: 2}) for 8000 merges: by default W = 5 untimed warmup
merges, then the remaining K = 7995 merges of the config are timed (every pass, tie pass and
exact pass of the run is inside the timed region).  Before the warmup merges, ~100 ms of plain count
passes over the resident corpus (no merge; --device-warmup-ms) bring the GPU to steady clocks.
With N > 1 GPUs each rank holds its own contiguous 1 GiB shard of one corpus stream (weak
scaling); the per-iteration pair-count exchange is an RCCL all-reduce enqueued on the engine's
stream between the selection and apply kernels (the rank loop, bpe-tokenizer_amd/sharded.py).

Prints ONE JSON line (rank 0), right after the timed region (the CPU baseline is measured before
any GPU work).  --incremental adds a second line: the same workload in the incremental mode.
"""
import argparse
import hashlib
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = json.load(open(os.path.join(ROOT, 'BASELINE.json')))['metric']
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
ALG_BYTES_PER_PAIR_SCAN = 4    # K1 reads each int32 token once


def cpu_model():
    try:
        for line in open('/proc/cpuinfo'):
            if line.startswith('model name'):
                return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return 'unknown'


def cpu_share():
    """The host cores this process may use, and why: the cgroup CPU quota (cgroup v2 cpu.max or
    v1 cfs_quota_us / cfs_period_us), the CPU affinity mask, and OMP_NUM_THREADS (the GPU pool sets
    it to the box's CPU share for one GPU and asks jobs to keep within it).  The multi-thread leg
    runs on the smallest of the three."""
    info = {'affinity': len(os.sched_getaffinity(0)), 'nproc': os.cpu_count()}
    quota = None
    try:
        q, p = open('/sys/fs/cgroup/cpu.max').read().split()[:2]
        info['cgroup_cpu_max'] = '%s %s' % (q, p)
        if q != 'max':
            quota = int(q) / int(p)
    except (OSError, ValueError):
        try:
            q = int(open('/sys/fs/cgroup/cpu/cpu.cfs_quota_us').read())
            p = int(open('/sys/fs/cgroup/cpu/cpu.cfs_period_us').read())
            info['cgroup_cfs_quota'] = '%d %d' % (q, p)
            if q > 0:
                quota = q / p
        except (OSError, ValueError):
            info['cgroup_cpu_max'] = 'unreadable'
    info['quota_cores'] = quota
    omp = int(os.environ.get('OMP_NUM_THREADS') or 0) or None
    info['omp_num_threads'] = omp
    limits = {'affinity': info['affinity']}
    if quota:
        limits['cgroup quota'] = max(1, int(quota))
    if omp:
        limits['OMP_NUM_THREADS (the pool\'s CPU share per GPU)'] = omp
    why = min(limits, key=limits.get)
    info['threads'] = limits[why]
    info['threads_bound_by'] = why
    return info


def cpu_baseline(sample_mib, budget_s, corpus='uniform'):
    """The multi-threaded CPU restatement (oracle/bpe_cpu_mt.cc: the same full recount per merge
    as the reference and the GPU engine, pinned to the reference's fixtures) on a bounded sample
    of the same workload, on all the host cores this process may use, then on one thread."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    from oracle import CpuMT
    pkg = importlib.import_module('bpe-tokenizer_amd')
    n = sample_mib << 20
    data = (pkg.synth_zipf(n, seed=12345) if corpus == 'zipf' else
            pkg.synth_latin1(n, seed=12345, A=256, base=0))
    lut = np.full(256, -1, np.int32)
    uniq, idx = np.unique(data, return_index=True)
    for k, u in enumerate(uniq[np.argsort(idx)]):
        lut[u] = k
    nt = int((lut >= 0).sum())
    ids = lut[data]
    del data
    off = np.arange(0, n + 1, 1 << 20, dtype=np.int64)
    share = cpu_share()
    threads = share['threads']

    def timed(T, budget):
        st = CpuMT(ids, off, [1] * nt, nt, threads=T, extra=1 << 14)
        scans = iters = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < budget or iters < 2:
            m = st.merge_until(0, 2, 1)
            if not m:
                break
            scans += st.last_scans
            iters += 1
        dt = time.perf_counter() - t0
        used = st.threads
        st.close()
        return scans / dt, iters, dt, used

    v_mt, it_mt, dt_mt, used = timed(threads, budget_s * 0.6)
    v_1, it_1, dt_1, _ = timed(1, budget_s * 0.4)
    return {'value': v_mt, 'unit': 'pair-scans/s', 'cores': used, 'kind': 'port',
            'value_1_thread': v_1,
            'host': dict(share, cpu_model=cpu_model()),
            'sample': '%d MiB of the same corpus stream (1 MiB samples), mergeUntil from the first '
                      'merge: %d merges in %.1f s on %d threads, %d merges in %.1f s on 1 thread; '
                      'oracle/bpe_cpu_mt.cc (full recount per merge, as the reference)'
                      % (sample_mib, it_mt, dt_mt, used, it_1, dt_1)}


def incremental_mode(args, stream_merges):
    """The same workload in the incremental mode (bpe_set_mode BPE_MODE_INCREMENTAL: mergeUntil on
    a position index, O(W) work per merge), on a fresh copy of the corpus:
    the W warmup merges untimed, then the K timed ones in one mergeUntil call, whose time includes
    the index build.  Reported apart from `value`, as the survey asks: its pair-scans are the
    reference's definition, not the work done.  The merge log must equal the streaming run's."""
    pkg = importlib.import_module('bpe-tokenizer_amd')
    n = args.corpus_mib << 20
    base = 0 if args.alphabet == 256 else 0x20
    data = (pkg.synth_zipf(n, seed=12345) if args.corpus == 'zipf' else
            pkg.synth_latin1(n, seed=12345, A=args.alphabet, base=base))
    e = pkg.Engine(0)
    e.add_latin1(data, sample_bytes=1 << 20)
    del data
    e.set_mode('incremental')
    e.merge_until(0, 2, args.warmup)
    live0 = e.corpus_size()[1]
    e.stats_enable(True)
    import torch
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    got = e.merge_until(0, 2, args.steps)
    dt = time.perf_counter() - t0
    scans, live = 0, live0
    for m in got:
        scans += live
        live -= m[2]
    st = e.stats()
    e.close()
    same = [tuple(map(int, m)) for m in got] == [tuple(map(int, m)) for m in stream_merges]
    return {'what': 'mergeUntil on the position index (csrc/bpe_pix.hip.h), one call of the K '
                    'timed merges, index build included',
            'ms_per_step': dt * 1e3 / max(1, len(got)), 'seconds': dt,
            'equiv_pair_scans_per_s': scans / dt, 'speedup_vs_stream_loop': None,
            'merges': len(got), 'identical_merges_to_stream': same,
            'index_builds': st['pix_builds'], 'index_build_ms': st['pix_build_ms'],
            'merges_on_index': st['pix_merges'],
            'handed_to_stream': st['pix_host']}


def encode_cpu_baseline(ids, off, abc, dev_out=None, dev_off=None, sample_texts=10000):
    """The device encoder's CPU baseline: the same rank-greedy algorithm on the host
    (oracle/bpe_cpu_encode.cc: a heap of (rank, position) per text, OpenMP over texts) over the
    same texts, on the host cores this process may use (cpu_share) and on one thread (a sample of
    the first texts).  With the device's output given, the CPU's must equal it on every text."""
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import oracle
    share = cpu_share()
    T = share['threads']
    oracle.cpu_encode_flat(ids, off[:2], abc, threads=1)   # (library load, rank table)
    t0 = time.perf_counter()
    got, oo, used = oracle.cpu_encode_flat(ids, off, abc, threads=T)
    t_mt = time.perf_counter() - t0
    k = min(sample_texts, len(off) - 1)
    t0 = time.perf_counter()
    oracle.cpu_encode_flat(ids, off[:k + 1], abc, threads=1)
    t_1 = time.perf_counter() - t0
    res = {'kind': 'port', 'cores': used, 'unit': 'tokens/s',
           'value': float(off[-1] - off[0]) / t_mt, 'seconds': t_mt,
           'value_1_thread': float(off[k] - off[0]) / t_1,
           'sample_1_thread': '%d texts, %d tokens, %.2f s' % (k, int(off[k] - off[0]), t_1),
           'what': 'oracle/bpe_cpu_encode.cc: the device encoder\'s rank-greedy algorithm on the '
                   'host (heap per text), all texts of the batch',
           'host': dict(share, cpu_model=cpu_model())}
    if dev_out is not None:
        res['identical_to_device'] = bool(np.array_equal(np.asarray(dev_off), oo) and
                                          np.array_equal(np.asarray(dev_out)[:oo[-1]], got))
    return res


def encode_line(args, merges, n_texts=100000, lo=16, hi=1024, reps=5):
    """encodeToCode (core.ts:392-409) of a batch of short texts on the device encoder, with the
    merge list the run made (the warmup merges + the timed ones): texts cut from a
    later, disjoint stretch of the same synthetic stream.  Kernel time (HIP events) and end to
    end time of bpe_encode_batch (its parity is the GPU tests' job: tests/test_encoder.py)."""
    pkg = importlib.import_module('bpe-tokenizer_amd')
    import numpy as np
    import time
    rng = np.random.default_rng(5)
    lens = rng.integers(lo, hi + 1, size=n_texts)
    need = int(lens.sum())
    n = args.corpus_mib << 20
    e = pkg.Engine(0)   # (the char map and the merges of the bench's own run: replayed here)
    data = (pkg.synth_zipf(n + need, seed=12345) if args.corpus == 'zipf' else
            pkg.synth_latin1(n + need, seed=12345, A=args.alphabet,
                             base=0 if args.alphabet == 256 else 0x20))
    cmap, n_tok, _ = e.add_latin1(data[:1 << 20], sample_bytes=1 << 20)
    e.close()
    ids = cmap[data[n:n + need]]
    ids = ids[ids >= 0].astype(np.int32)
    off = np.zeros(n_texts + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    off = np.minimum(off, ids.size)
    abc = np.asarray([(a, b, n_tok + k) for k, (a, b, _w) in enumerate(merges)], np.int32)
    enc = pkg.Encoder(0, abc)
    enc.encode_flat(ids, off)
    enc.reset_stats()
    t0 = time.perf_counter()
    for _ in range(reps):
        out, oo = enc.encode_flat(ids, off)
    e2e = (time.perf_counter() - t0) / reps
    st = enc.stats()
    enc.close()
    kern = st['kernel_ms'] / reps / 1e3
    return {'what': 'encodeToCode of %d texts of %d-%d chars on the device encoder, the %d merges '
                    'of the timed run' % (n_texts, lo, hi, len(merges)),
            'tokens_in': int(off[-1]), 'tokens_out': int(oo[-1]),
            'kernel_ms': kern * 1e3, 'e2e_ms': e2e * 1e3,
            'kernel_tokens_per_s': off[-1] / kern, 'e2e_tokens_per_s': off[-1] / e2e,
            'steps_per_text': st['steps'] / reps / n_texts,
            'cpu_baseline': encode_cpu_baseline(ids, off, abc, out, oo)}


def maintained_roofline(st, traffic):
    """Roofline of the device loop's maintained-state passes alone (k_step_loop<MODE_INCR>, the
    stats' incr_* fields: HIP events over every 8th iteration, live tokens over all of them), or
    None when the run made none."""
    if not st.get('incr_timed'):
        return None
    k_ms = st['incr_ms'] / st['incr_timed']
    alg = ALG_BYTES_PER_PAIR_SCAN * st['incr_live'] / max(1, st['incr_launches'])
    achieved = alg / (k_ms * 1e-3) / 1e9
    out = {'bound': 'hbm', 'kernel': 'k_step_loop<MODE_INCR> (apply + recount of the pairs '
                                     'touching the merge)',
           'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
           'frac': achieved / HBM_PEAK_GBS, 'kernel_avg_ms': k_ms, 'launches': st['incr_launches'],
           'alg_bytes_per_launch': alg, 'traffic': None}
    if 'MODE_INCR' in str(traffic.get('kernel', '')) or traffic.get('kernel') == 'k_step_loop<4>':
        out['traffic'] = traffic.get('traffic_bytes_per_launch')
        out['traffic_source'] = traffic.get('source')
    return out


def device_warmup(trainer, ms):
    """Plain count passes over the resident corpus (bpe_recount: no merge, the corpus and the merge
    sequence are unchanged) for about `ms` ms before the W warmup merges.  A fresh box's first
    passes run slower (clocks and caches coming up: profiles/r06_warm_probe.jsonl, the first ~10
    launches 780-840 us against 755 us after), and the driver's W = 5 warmup merges are ~4 ms of
    GPU work; so the timed window starts at steady state, as the full run's does.  Outside the
    timed region; reported in the line (`device_warmup`)."""
    import torch
    if ms <= 0:
        return None
    eng = trainer.engine
    t0 = time.perf_counter()
    n = 0
    while True:
        for _ in range(8):
            eng.recount()
        n += 8
        torch.cuda.synchronize()
        if (time.perf_counter() - t0) * 1e3 >= ms:
            break
    return {'count_passes': n, 'seconds': time.perf_counter() - t0,
            'what': 'plain count passes (bpe_recount) over the resident corpus before the warmup '
                    'merges; no merge, corpus unchanged'}


def fixture_check(args, merges):
    """The run's merge list against the threaded CPU restatement's run of the same workload
    (tests/golden/config3_cpu_mt_8000.json for C3, zipf_cpu_mt_2000.json for the skewed variant;
    oracle/gen_cpu_mt_fixtures.py): the first min(len) merges must be equal.  None when no
    fixture covers this workload (another corpus size or alphabet)."""
    if args.corpus_mib != 1024 or (args.corpus == 'uniform' and args.alphabet != 256):
        return None
    name = 'config3_cpu_mt_8000.json' if args.corpus == 'uniform' else 'zipf_cpu_mt_2000.json'
    path = os.path.join(ROOT, 'tests', 'golden', name)
    if not os.path.exists(path):
        return None
    want = json.load(open(path))['merges']
    n = min(len(want), len(merges))
    got = [list(map(int, m)) for m in merges[:n]]
    return {'fixture': 'tests/golden/' + name, 'merges_compared': n,
            'merges_match_fixture': got == want[:n]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=7995)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--corpus-mib', type=int, default=1024, help='corpus MiB per GPU')
    ap.add_argument('--alphabet', type=int, default=256)
    ap.add_argument('--corpus', choices=['uniform', 'zipf'], default='uniform',
                    help='uniform: the C3 byte stream; zipf: the skewed variant (Zipf 1.1 words)')
    ap.add_argument('--cpu-sample-mib', type=int, default=256)
    ap.add_argument('--cpu-budget-s', type=float, default=20.0)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--device-warmup-ms', type=float, default=100.0,
                    help='plain count passes over the resident corpus (no merge) before the warmup '
                         'merges, so that the timed window starts at steady clocks (0: none)')
    ap.add_argument('--incremental', action='store_true',
                    help='also run the incremental mode on the same workload, printed as a second '
                         'JSON line after the bench line')
    ap.add_argument('--encode', action='store_true',
                    help='also run the device encoder (encodeToCode, bpe_encode_batch) with the '
                         'merges of the timed run over 100 000 texts of 16-1024 chars of the same '
                         'stream, printed as a further JSON line')
    args = ap.parse_args()

    import torch
    rank = int(os.environ.get('RANK', '0'))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus:
        raise SystemExit('--gpus %d but WORLD_SIZE=%d' % (args.gpus, world))
    # the CPU baseline first (host cores only, before any GPU work), so that nothing but the print
    # follows the timed region
    cpu = None
    if world == 1 and rank == 0 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_sample_mib, args.cpu_budget_s, args.corpus)
    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group('nccl', device_id=torch.device('cuda', local_rank))

    pkg = importlib.import_module('bpe-tokenizer_amd')
    from importlib import import_module
    sharded = import_module('bpe-tokenizer_amd.sharded')

    n = args.corpus_mib << 20
    base = 0 if args.alphabet == 256 else 0x20
    trainer = sharded.ShardedTrainer.synthetic(device=local_rank, rank=rank, world=world,
                                               bytes_per_rank=n, sample_bytes=1 << 20,
                                               seed=12345, alphabet=args.alphabet, base=base,
                                               dist=dist, corpus=args.corpus)

    heat = device_warmup(trainer, args.device_warmup_ms)
    if len(trainer.run(args.warmup, max_length=0, min_weight=2)) != args.warmup:
        raise SystemExit('corpus exhausted during warmup')
    trainer.engine.reset_stats()
    trainer.engine.stats_enable(True)
    live0 = trainer.live_tokens_global()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    merges = trainer.run(args.steps, max_length=0, min_weight=2)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    if len(merges) != args.steps:
        raise SystemExit('corpus exhausted before the timed steps finished')
    # pair-scans: every iteration scans the live corpus it starts from
    scans = 0
    live = live0
    for m in merges:
        scans += live
        live -= m[2]
    if dist:
        t = torch.tensor([dt], dtype=torch.float64, device='cuda')
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    st = trainer.engine.stats()

    if rank == 0:
        # HBM bytes per launch of the same kernel from rocprofv3 FETCH_SIZE / WRITE_SIZE passes over
        # this same command (tools/gpu_round.sh -> tools/pmc_summary.py; counters cannot be read
        # from inside the timed run)
        traffic = {}
        tpath = os.path.join(ROOT, 'profiles', 'current_pmc.json' if args.corpus == 'uniform'
                             else 'current_pmc_%s.json' % args.corpus)
        if os.path.exists(tpath):
            # (each corpus has its own committed passes: tools/gpu_round2.sh, tools/zipf_prof.sh)
            traffic = json.load(open(tpath))
        # (the device loop times every 8th iteration: step_ms and select_ms cover step_timed passes)
        k1_ms = st['step_ms'] / max(1, st['step_timed'])
        timed_frac = st['step_timed'] / max(1, st['step_launches'])
        live_per_launch = st['step_live'] / max(1, st['step_launches'])
        slots_per_launch = st['step_slots'] / max(1, st['step_launches'])
        achieved = ALG_BYTES_PER_PAIR_SCAN * live_per_launch / (k1_ms * 1e-3) / 1e9
        out = {
            'metric': METRIC,
            'value': scans / dt,
            'unit': 'pair-scans/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': dt * 1e3 / args.steps,
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'int32',
            'data': 'synthetic',
            'config': {
                'workload': (('C3: %d MiB/GPU latin1 corpus, xorshift32 seed 12345, %d-char '
                              'alphabet' % (args.corpus_mib, args.alphabet))
                             if args.corpus == 'uniform' else
                             ('C3-zipf (skewed variant): %d MiB/GPU of Zipf(1.1) words over a '
                              '32768-word list, seed 12345' % args.corpus_mib))
                            + '; 1 MiB samples; merges %d..%d of mergeUntil({min_weight:2})'
                            % (args.warmup + 1, args.warmup + args.steps),
                'corpus_tokens': live0,
                'parallelism': 'corpus-sharded x%d' % world,
            },
            'roofline': {
                'bound': 'hbm',
                'kernel': ('k_step (fused K4 apply + K1 pair count, one pass per merge)'
                           if args.corpus == 'uniform' else
                           'k_step (fused K4 apply + K1 pair count; in the maintained state '
                           'k_step_loop<MODE_INCR>: apply + recount of the pairs touching the merge)'),
                'achieved': achieved,
                'peak': HBM_PEAK_GBS,
                'unit': 'GB/s',
                'frac': achieved / HBM_PEAK_GBS,
                'traffic': traffic.get('traffic_bytes_per_launch'),
                'kernel_avg_ms': k1_ms,
                'alg_bytes_per_launch': ALG_BYTES_PER_PAIR_SCAN * live_per_launch,
                'slots_streamed_per_launch': slots_per_launch,
                'traffic_fetch_bytes': traffic.get('fetch_bytes_per_launch'),
                'traffic_write_bytes': traffic.get('write_bytes_per_launch'),
                'traffic_source': traffic.get('source'),
            },
            # (the maintained state's passes on their own: the skewed corpus's pass once its
            # table state is left, the kernel the zipf counters in current_pmc_zipf.json are of)
            'roofline_maintained_pass': maintained_roofline(st, traffic),
            # (identity of the run's merge list across builds and modes: sha256 of the (a, b, W)
            # triples as int64, warmup merges included)
            'merges_sha256': hashlib.sha256(
                np.asarray(trainer.merges, dtype=np.int64).tobytes()).hexdigest(),
            # (the merges of the whole run, warmup included, against the CPU restatement's run)
            'fixture_check': fixture_check(args, trainer.merges) if world == 1 else None,
            'device_warmup': heat,
            'breakdown_ms_per_step': {
                'stream_pass': k1_ms * st['step_launches'] / max(1, args.steps),
                'select': st['select_ms'] / max(1e-9, timed_frac) / max(1, args.steps),
                'tie_passes': st['tie_passes'],
                'compactions': st['compactions'],
                'exact_passes': st['exact_passes'], 'cold_rebuilds': st['cold_rebuilds'],
                # (passes whose LDS adds return nothing: no counter can reach 16 bits, LoopCtl::
                # unscreened in csrc/bpe_kernels.hip.h)
                'unscreened_passes': st.get('unscreened_passes'),
            },
        }
        if cpu is not None:
            out['cpu_baseline'] = cpu
        print(json.dumps(out), flush=True)
        if world == 1 and args.incremental:
            trainer.engine.close()
            inc = incremental_mode(args, merges)
            inc['speedup_vs_stream_loop'] = (dt * 1e3 / args.steps) / inc['ms_per_step']
            print(json.dumps({'incremental_mode': inc}), flush=True)
        if world == 1 and args.encode:
            print(json.dumps({'encode': encode_line(args, trainer.merges)}), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
