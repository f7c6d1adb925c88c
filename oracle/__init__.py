"""ORACLE — CPU fp64 restatement of the reference's hot path, used ONLY as the
checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
Never imported by the product (franka-force-feedback-mpc_amd/ffddp)."""
