"""TEST INFRASTRUCTURE: CPU oracle of the blockwise DT watershed (see ctws_oracle.cpp).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.
"""
