"""CPU oracle of the DGP-RF SGHMC/SGLD hot path — TEST INFRASTRUCTURE ONLY.

May be imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
checker / CPU baseline — never by the product (dgp-rf-mcmc_amd/).  Parity status: see
oracle/dgp_oracle.py (unpinned against the reference's outputs; pinned by the reference's printed
known answers, torch autograd and the Random123 KATs).
"""
