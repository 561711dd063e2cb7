"""``kdl`` command line: manager daemon, kubectl-like client, one-shot runs, benchmarks."""
