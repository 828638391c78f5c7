"""Diagnostic: SGHMC steps of config 2 in N processes sharing one GPU (what the two-rank gloo
bench rehearsal does), W-only and full-Bayes, each phase started together through a file barrier.

  python scripts/diag/coresident.py [nproc] [steps] [steps_per_graph]

The parent never touches the GPU; it starts the workers as child processes and prints their
lines.  Each worker prints µs/step of its own graph replays, per phase."""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def barrier(tag, rank, n, phase):
    open(f"/tmp/coresident_{tag}_{phase}_{rank}", "w").close()
    while not all(os.path.exists(f"/tmp/coresident_{tag}_{phase}_{r}") for r in range(n)):
        time.sleep(0.0005)


def worker(tag, rank, n, steps, spg):
    import torch
    sys.path[:0] = [ROOT, os.path.join(ROOT, "dgp-rf-mcmc_amd")]
    from dgprf import engine as E
    from dgprf.data import CONFIGS, regression_data
    from likelihoods import Gaussian
    from models.dgp import DGP_RF
    c = CONFIGS[2]
    dev = torch.device("cuda", 0)
    X, Y, _ = regression_data(c["n"], c["d_in"], seed=0, device=dev)
    E.set_seed(3 + rank)
    m = DGP_RF(c["d_in"], c["d_out"], n_hidden_layers=len(c["kinds"]), n_rf=c["n_rf"],
               n_gp=c["n_gp"], likelihood=Gaussian(variance=c["variance"]),
               kernel_type_list=c["kinds"])
    run = dict(batch_size=c["batch"], lr=c["lr"], momentum_decay=c["beta"], temperature=c["T"],
               steps_per_graph=spg)
    m.precond_update(None, c["n"], precond_type="identity")
    m.run_sgmcmc(X, Y, c["n"], 2 * spg, **run)
    m.precond_update(None, c["n"], precond_type="identity", full_bayesian=True)
    m.run_sgmcmc(X, Y, c["n"], 2 * spg, full_bayesian=True, **run)
    torch.cuda.synchronize()
    out = []
    for phase, fb in (("w", False), ("fb", True), ("w2", False), ("fb2", True)):
        barrier(tag, rank, n, phase)
        t0 = time.perf_counter()
        m.run_sgmcmc(X, Y, c["n"], steps, full_bayesian=fb, **run)
        torch.cuda.synchronize()
        out.append(f"{phase} {(time.perf_counter() - t0) * 1e6 / steps:.1f}")
    print(f"rank {rank}/{n}: us/step " + ", ".join(out), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--worker":
        worker(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), int(sys.argv[6]))
        return 0
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    spg = int(sys.argv[3]) if len(sys.argv) > 3 else 100
    tag = f"{os.getpid()}"
    procs = [subprocess.Popen([sys.executable, "-u", __file__, "--worker", tag, str(r), str(n),
                               str(steps), str(spg)]) for r in range(n)]
    rc = 0
    for p in procs:
        rc |= p.wait()
    for f in os.listdir("/tmp"):
        if f.startswith(f"coresident_{tag}_"):
            os.remove(os.path.join("/tmp", f))
    return rc


if __name__ == "__main__":
    sys.exit(main())
