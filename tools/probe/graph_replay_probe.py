"""Per-node cost of a replayed HIP graph on this ROCm: a chain of N tiny dependent kernels
(x.add_(1) on 1 Ki floats) captured once, replayed back to back -- device time per replay
(events) and per node, against the same chain launched eagerly.  The NER update is ~220
kernels: if a replay costs far more than its kernels, the graph runtime (not the host, not the
kernels) bounds it.  ``python tools/probe/graph_replay_probe.py [--nodes 220]``; try it under the
runtime's DEBUG_CLR_GRAPH_PACKET_CAPTURE / DEBUG_HIP_GRAPH_BATCH_SIZE settings."""
import argparse
import json
import os
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--nodes', type=int, default=220)
    ap.add_argument('--reps', type=int, default=50)
    ap.add_argument('--numel', type=int, default=1024, help='floats per kernel (dirty bytes per node)')
    a = ap.parse_args()
    x = torch.zeros(a.numel, device='cuda')
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            for _ in range(a.nodes):
                x.add_(1.0)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(a.nodes):
            x.add_(1.0)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(a.reps):
        g.replay()
    e1.record()
    e1.synchronize()
    t_graph = e0.elapsed_time(e1) / a.reps
    host_graph = (time.perf_counter() - t0) * 1e3 / a.reps
    t0 = time.perf_counter()
    e0.record()
    for _ in range(a.reps):
        for _ in range(a.nodes):
            x.add_(1.0)
    e1.record()
    e1.synchronize()
    t_eager = e0.elapsed_time(e1) / a.reps
    host_eager = (time.perf_counter() - t0) * 1e3 / a.reps
    env = {k: v for k, v in os.environ.items() if k.startswith(('DEBUG_CLR', 'DEBUG_HIP'))}
    print(json.dumps({'nodes': a.nodes, 'numel': a.numel, 'env': env, 'graph_ms': round(t_graph, 3),
                      'graph_us_per_node': round(t_graph * 1e3 / a.nodes, 2), 'graph_host_ms': round(host_graph, 3),
                      'eager_ms': round(t_eager, 3), 'eager_us_per_kernel': round(t_eager * 1e3 / a.nodes, 2),
                      'eager_host_ms': round(host_eager, 3)}), flush=True)


if __name__ == '__main__':
    main()
