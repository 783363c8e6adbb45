"""Merge TunableOp CSV dumps into the shipped table:
``python tools/merge_gemm_tables.py OUT.csv IN1.csv [IN2.csv ...]``."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hetseq_9cme_amd.ops.gemm_tuning import merge_tables  # noqa: E402

if __name__ == '__main__':
    print(merge_tables(sys.argv[2:], sys.argv[1]), 'rows')
