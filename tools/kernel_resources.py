"""Per-kernel register / spill / LDS summary of one .hip translation unit (hipcc
-Rpass-analysis=kernel-resource-usage), for checking a kernel before it goes to the GPU.
Usage: python tools/kernel_resources.py hetseq_9cme_amd/csrc/kernels/gemm_f16.hip [name-filter]"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ''
    out = os.path.join(tempfile.gettempdir(), 'hx_kr.o')
    r = subprocess.run(['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-c', src, '-o', out,
                        '-I' + os.path.join(ROOT, 'hetseq_9cme_amd', 'csrc', 'include'), '-munsafe-fp-atomics',
                        '-Rpass-analysis=kernel-resource-usage'], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                       text=True)
    cur, rows = None, []
    for line in r.stdout.splitlines():
        m = re.search(r'Function Name: (\S+)', line)
        if m:
            cur = {'name': m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r'remark: +(VGPRs|AGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)', line)
        if m and cur is not None:
            cur[m.group(1).split(' [')[0]] = int(m.group(2))
    if r.returncode:
        print(r.stdout[-3000:])
    for d in rows:
        if filt in d['name']:
            print('{:>4} V {:>4} A  spill {:>3}/{:<3} occ {:>2} lds {:>6}  {}'.format(
                d.get('VGPRs', -1), d.get('AGPRs', -1), d.get('VGPRs Spill', -1), d.get('SGPRs Spill', -1),
                d.get('Occupancy', -1), d.get('LDS Size', -1), d['name'][:110]))


if __name__ == '__main__':
    main()
