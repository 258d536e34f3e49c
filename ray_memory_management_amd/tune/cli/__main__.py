"""``python -m ray_memory_management_amd.tune.cli {ls,lsx} PATH [options]``."""
import argparse
import sys

from ray_memory_management_amd.tune.cli.commands import list_experiments, list_trials


def main(argv=None):
    ap = argparse.ArgumentParser(prog="tune")
    sub = ap.add_subparsers(dest="cmd", required=True)
    for name, help_ in (("ls", "list the trials of an experiment"), ("lsx", "list the experiments of a project")):
        p = sub.add_parser(name, help=help_)
        p.add_argument("path")
        p.add_argument("--sort", action="append")
        p.add_argument("--output", "-o")
        p.add_argument("--filter", dest="filter_op", help="'<column> <op> <value>', e.g. 'score > 0.5'")
        p.add_argument("--columns", help="comma-separated columns")
        p.add_argument("--limit", type=int)
        p.add_argument("--desc", action="store_true")
    a = ap.parse_args(argv)
    fn = list_trials if a.cmd == "ls" else list_experiments
    print(fn(a.path, a.sort, a.output, a.filter_op, a.columns.split(",") if a.columns else None, a.limit, a.desc))
    return 0


if __name__ == "__main__":
    sys.exit(main())
