"""Local rehearsal of a heterogeneous multi-node HetSeq launch on ONE machine.

Each "node" is a separate launcher process that owns a disjoint subset of the
local GPUs and passes ``--distributed-gpus g_n --distributed-rank r_n`` exactly
like the per-node qsub/ssh scripts of the reference (STORE_RUN_FILE/Train_mnist/*_het);
all nodes meet through one TCP rendezvous on 127.0.0.1.  Example (the BASELINE 5+3
split on an 8-GPU box):

  python tools/launch_hetero.py --nodes 5,3 -- --task bert --data D --config_file C \
      --max-sentences 128 --fast-stat-sync --max-update 100

GPU ownership: by default (``--device-offset``) every launcher sees ALL GPUs and its ranks
run on GPUs offset .. offset + g_n - 1 (train.py ``--device-offset``), so the ranks of
different "nodes" can still map each other's memory -- the hand-written xGMI transport
(--allreduce-impl xgmi) works across the split.  ``--partition`` instead hides the other
nodes' GPUs with HIP_VISIBLE_DEVICES (closest to separate machines; RCCL only).
"""
import argparse
import os
import random
import subprocess
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--nodes', default='5,3', help='comma separated GPU count per "node"')
    ap.add_argument('--port', type=int, default=0)
    ap.add_argument('--cpu', action='store_true', help='gloo on CPU (no GPU partitioning)')
    ap.add_argument('--partition', action='store_true',
                    help='HIP_VISIBLE_DEVICES per node instead of --device-offset (peers invisible)')
    ap.add_argument('rest', nargs=argparse.REMAINDER)
    a = ap.parse_args()
    rest = a.rest[1:] if a.rest and a.rest[0] == '--' else a.rest
    counts = [int(x) for x in a.nodes.split(',')]
    world = sum(counts)
    port = a.port or random.randint(20000, 30000)
    init = 'tcp://127.0.0.1:{}'.format(port)
    procs, base, dev0 = [], 0, 0
    for g in counts:
        env = dict(os.environ)
        cmd = [sys.executable, '-m', 'hetseq_9cme_amd.train'] + rest + [
            '--distributed-init-method', init, '--distributed-world-size', str(world),
            '--distributed-gpus', str(g), '--distributed-rank', str(base)]
        if not a.cpu and a.partition:
            env['HIP_VISIBLE_DEVICES'] = ','.join(str(d) for d in range(dev0, dev0 + g))
        elif not a.cpu:
            cmd += ['--device-offset', str(dev0)]
        if a.cpu:
            cmd += ['--cpu']
        if g == 1:
            cmd += ['--distributed-no-spawn']
        procs.append(subprocess.Popen(cmd, env=env))
        base += g
        dev0 += g
    rc = 0
    for p in procs:
        rc = p.wait() or rc
    sys.exit(rc)


if __name__ == '__main__':
    main()
