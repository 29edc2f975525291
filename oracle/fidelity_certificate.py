"""Fidelity certificate of the CPU restatement — build container only.

    python oracle/fidelity_certificate.py [--threads 8] [--reps 3]

Times the oracle (oracle/flows_ref.py, the restatement bench.py's cpu_baseline runs on the GPU
box's host) against the reference implementation itself (imported from /root/reference with the
same torchdiffeq stub as tests/golden/make_golden.py) on identical inputs and weights: eval
log_prob (inverse + MultivariateNormal base term) at B = 1M for cfg2, cfg3 and cfg4 (5x MAF(63,64),
1M of its 4M rows). Prints one JSON object: per config the median wall time of both, their ratio
(the certificate asks for oracle/reference within +-10 %), and the NLL of both (must agree).
The reference never leaves this container; only the numbers are recorded.
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

import oracle  # noqa: E402
from make_golden import import_reference, mvn_logp, perturb, spline_stack, maf_stack  # noqa: E402


def timed(fn, reps):
    with torch.no_grad():
        out = fn()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
    return statistics.median(ts), out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    flows, models = import_reference()
    res = {"threads": a.threads, "torch": torch.__version__, "reps": a.reps}

    torch.manual_seed(0)
    m2 = models.RealNVP(2, 8, 64)
    perturb(m2, 0.1, 1)
    m3 = spline_stack(flows, models, 2, 64, 8, 8, 10)
    perturb(m3, 0.1, 11)
    m5 = maf_stack(flows, models, 63, 64, 5, 30)
    perturb(m5, 0.02, 31)
    cases = [("cfg2", m2, 2, 1234, oracle.realnvp_spec(8)),
             ("cfg3", m3, 2, 1235, [("spline", f"flows.{i}.", {"K": 8}) for i in range(8)]),
             ("cfg4", m5, 63, 1236, oracle.maf_spec(5))]
    for name, m, d, seed, spec in cases:
        m.eval()
        x = torch.randn(1_000_000, d, generator=torch.Generator().manual_seed(seed))
        sd = {k: v.detach().clone() for k, v in m.state_dict().items()}

        def ref():
            z, ld = m.inverse(x)
            return mvn_logp(z, ld)

        def port():
            z, ld = oracle.flow_model(sd, spec, x, -1)
            return oracle.gauss_log_prob(z, ld)

        t_ref, lp_ref = timed(ref, a.reps)
        t_port, lp_port = timed(port, a.reps)
        res[name] = {"B": 1_000_000, "reference_s": t_ref, "oracle_s": t_port, "oracle_over_reference": t_port / t_ref,
                     "within_10pct": abs(t_port / t_ref - 1) <= 0.10,
                     "nll_reference": -float(lp_ref.double().mean()), "nll_oracle": -float(lp_port.double().mean())}
        print(name, res[name], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
