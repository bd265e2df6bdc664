"""CPU oracle — test infrastructure only (see kge_oracle.py header).

Never imported by knowledgegraphembedding_amd; only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
