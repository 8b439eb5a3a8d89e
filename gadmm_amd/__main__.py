"""``python -m gadmm_amd <Entry> [options]`` — run a reference experiment.

Entries: LinearRegression_Synthetic, LinearRegression_Real, LogisticRegression_Synthetic,
LogisticRegression_Real, Dynamic_LinearRegression_Synthetic, Dynamic_LinearRegression_Real,
LinearRegression_gadmm_vs_admm, LinearRegression_RealShaped (10M x 10k sharded, MI355X).
``python -m gadmm_amd list`` shows them; ``python -m gadmm_amd <Entry> -h`` the options.
"""
import sys


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    from . import entry

    if not argv or argv[0] in ("-h", "--help", "list"):
        print(__doc__)
        for e in entry.ENTRIES:
            print("  ", e)
        return 0
    mod = entry.get(argv[0])
    mod.main(argv[1:])
    return 0


if __name__ == "__main__":
    sys.exit(main())
