"""TEST INFRASTRUCTURE ONLY — CPU restatements of the reference algorithms on the hot path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package,
and only as the checker / the timed CPU baseline. The product (transplat_amd) never imports it.
Each restatement cites the reference file:line it follows; see DESIGN.md §Oracle for what is
pinned by golden vectors generated from the reference and what is "parity unpinned".
"""
