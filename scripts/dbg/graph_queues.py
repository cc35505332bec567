"""How a captured multi-stream schedule executes: the SDR stack's stream patterns with
spin kernels (torch.cuda._sleep) standing in for its launches, captured in a hipGraph
and replayed; prints each pattern's replay time against its critical-path bound and
the eager time.  Under rocprofv3 --kernel-trace the spin kernels' Queue_Id show which
hardware queue each logical stream's nodes landed on (durations tag the streams:
A ~1x, B ~2x, C ~0.5x the unit).
    python scripts/dbg/graph_queues.py [--unit 20000] [--K 20]"""
import argparse
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--unit', type=int, default=200000, help='spin cycles of one A node')
    ap.add_argument('--K', type=int, default=20)
    ap.add_argument('--reps', type=int, default=5)
    a = ap.parse_args()
    dev = torch.device('cuda:0')
    U, K = a.unit, a.K
    ss = {n: torch.cuda.Stream(device=dev) for n in 'ABC'}

    def spin(s, mult):
        with torch.cuda.stream(s):
            torch.cuda._sleep(int(U * mult))

    def fwd_cur():
        """forward as shipped: A diag d; C pose(k) after A's d - 1; B fwd(k) after C."""
        A, B, C = ss['A'], ss['B'], ss['C']
        ev_a = [torch.cuda.Event() for _ in range(K + 1)]
        ev_p = [torch.cuda.Event() for _ in range(K)]
        for d in range(K + 1):
            if d < K:
                spin(A, 1.0)
            ev_a[d].record(A)
            k = d - 1
            if k >= 0:
                C.wait_event(ev_a[d - 1])
                spin(C, 0.5)
                ev_p[k].record(C)
                B.wait_event(ev_p[k])
                spin(B, 2.0)

    def fwd_pose_on_a():
        """pose(k) on A right after diag k, then B fwd(k) after A."""
        A, B = ss['A'], ss['B']
        ev = [torch.cuda.Event() for _ in range(K)]
        for d in range(K):
            spin(A, 1.0)
            spin(A, 0.5)
            ev[d].record(A)
            B.wait_event(ev[d])
            spin(B, 2.0)

    def fwd_pose_on_a_deferred():
        """as fwd_pose_on_a, but B's launch captured after A's next node."""
        A, B = ss['A'], ss['B']
        ev = [torch.cuda.Event() for _ in range(K)]
        for d in range(K + 1):
            if d < K:
                spin(A, 1.0)
                spin(A, 0.5)
                ev[d].record(A)
            if d >= 1:
                B.wait_event(ev[d - 1])
                spin(B, 2.0)

    def bwd_side():
        """backward as shipped now: B rec(k); C gxw(k) after B; A diag after C."""
        A, B, C = ss['A'], ss['B'], ss['C']
        ev_r = [torch.cuda.Event() for _ in range(K)]
        ev_b = [torch.cuda.Event() for _ in range(K)]
        for k in range(K):
            spin(B, 2.0)
            ev_r[k].record(B)
            C.wait_event(ev_r[k])
            spin(C, 0.5)
            ev_b[k].record(C)
            A.wait_event(ev_b[k])
            spin(A, 1.0)

    def bwd_inline():
        """backward of round 4: B rec(k) + gxw(k); A diag after B."""
        A, B = ss['A'], ss['B']
        ev_b = [torch.cuda.Event() for _ in range(K)]
        for k in range(K):
            spin(B, 2.0)
            spin(B, 0.5)
            ev_b[k].record(B)
            A.wait_event(ev_b[k])
            spin(A, 1.0)

    def bwd_gxw_on_a():
        """B rec(k) only; A runs gxw(k) then its diag after B's rec(k)."""
        A, B = ss['A'], ss['B']
        ev = [torch.cuda.Event() for _ in range(K)]
        for k in range(K):
            spin(B, 2.0)
            ev[k].record(B)
            A.wait_event(ev[k])
            spin(A, 0.5)
            spin(A, 1.0)

    def bwd_gxw_on_a_deferred():
        """as bwd_gxw_on_a, A's nodes captured after B's next launch."""
        A, B = ss['A'], ss['B']
        ev = [torch.cuda.Event() for _ in range(K)]
        for k in range(K + 1):
            if k < K:
                spin(B, 2.0)
                ev[k].record(B)
            if k >= 1:
                A.wait_event(ev[k - 1])
                spin(A, 0.5)
                spin(A, 1.0)

    pats = [('fwd_cur', fwd_cur, 0.5 + 2.0 * K + 1.0), ('fwd_pose_on_a', fwd_pose_on_a, 1.5 + 2.0 * K),
            ('fwd_pose_on_a_deferred', fwd_pose_on_a_deferred, 1.5 + 2.0 * K),
            ('bwd_side', bwd_side, 2.0 * K + 1.5), ('bwd_inline', bwd_inline, 2.5 * K + 1.0),
            ('bwd_gxw_on_a', bwd_gxw_on_a, 2.0 * K + 1.5),
            ('bwd_gxw_on_a_deferred', bwd_gxw_on_a_deferred, 2.0 * K + 1.5)]
    # unit time: one A node alone
    torch.cuda._sleep(U)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        torch.cuda._sleep(U)
    e1.record()
    torch.cuda.synchronize()
    unit = e0.elapsed_time(e1) / 20
    print('unit (one A node) %.1f us' % (unit * 1e3))
    for name, fn, bound in pats:
        def body():
            main = torch.cuda.current_stream(dev)   # the capture stream inside torch.cuda.graph
            for s_ in ss.values():
                s_.wait_stream(main)
            fn()
            for s_ in ss.values():
                main.wait_stream(s_)
        body()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.reps):
            body()
        torch.cuda.synchronize()
        eager = (time.perf_counter() - t) / a.reps * 1e3
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            body()
        g.replay()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.reps):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        gt = e0.elapsed_time(e1) / a.reps
        print('%-24s bound %7.2f ms  graph %7.2f ms (%.2fx)  eager %7.2f ms' %
              (name, bound * unit, gt, gt / (bound * unit), eager))


if __name__ == '__main__':
    main()
