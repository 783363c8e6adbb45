"""Regenerate docs/parameters.md from the live argument parser:
``python tools/gen_parameters_doc.py > docs/parameters.md``."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hetseq_9cme_amd import options  # noqa: E402

NEW = {'--async-save', '--check-params-every', '--distributed-timeout', '--ent_name_id_file', '--fused-kernels',
       '--gemm-tuning', '--gemm-tuning-file', '--precision', '--profile-phases', '--user-module',
       '--overlap-wgrad', '--no-overlap-wgrad', '--debug-kernels', '--allreduce-impl', '--xgmi-blocks', '--device-offset',
       '--bucket-peer-mb', '--comm-cus', '--force-reducer', '--fp32-gemm', '--graph-train-step',
       '--pad-to-multiple-of', '--rccl-normal-priority'}

SECTIONS = [('bert', 'adam'), ('mnist', 'adadelta'), ('BertForTokenClassification', 'adam'),
            ('BertForELClassification', 'adam')]


def rows(parser):
    seen = []
    for g in parser._action_groups:
        for a in g._group_actions:
            if isinstance(a, argparse._HelpAction) or not a.option_strings:
                continue
            seen.append((g.title or '', a))
    return seen


def fmt_flag(a):
    return '`{}`{}'.format(', '.join(a.option_strings), ' *(new)*' if a.option_strings[0] in NEW else '')


def fmt_default(a):
    if isinstance(a, argparse._StoreTrueAction):
        return 'on' if a.default else 'off'
    if isinstance(a, argparse._StoreFalseAction):
        return 'off' if a.default else 'on'
    if isinstance(a, argparse._StoreConstAction) and a.const is not None:
        return '`{}`'.format(a.default) if a.default is not None else '—'
    return '`{}`'.format(a.default) if a.default is not None else '—'


def main():
    print('# Command-line parameters\n')
    print('Generated from `hetseq_9cme_amd/options.py` by `tools/gen_parameters_doc.py`. Names and defaults '
          'match the original HetSeq flags (reference `hetseq/options.py`); flags marked *(new)* are '
          'MI355X-native additions.  Task / optimizer / LR-scheduler specific flags appear only when that '
          'choice is selected (two-phase parse, like the reference).\n')
    base_names = None
    for task, opt in SECTIONS:
        p = options.get_training_parser(task=task, optimizer=opt)
        rs = rows(p)
        names = {a.option_strings[0] for _, a in rs}
        if base_names is None:
            print('## Common flags (shown with `--task bert --optimizer adam`)\n')
            print('| flag | default | group | help |')
            print('|---|---|---|---|')
            for title, a in rs:
                print('| {} | {} | {} | {} |'.format(fmt_flag(a), fmt_default(a), title,
                                                     (a.help or '').replace('|', '/').replace('\n', ' ')))
            base_names = names
            print()
            continue
        extra = [(t, a) for t, a in rs if a.option_strings[0] not in base_names]
        print('## Additional flags with `--task {}` / `--optimizer {}`\n'.format(task, opt))
        print('| flag | default | help |')
        print('|---|---|---|')
        for _, a in extra:
            print('| {} | {} | {} |'.format(fmt_flag(a), fmt_default(a),
                                             (a.help or '').replace('|', '/').replace('\n', ' ')))
        print()


if __name__ == '__main__':
    main()
