"""Long randomized GPU-vs-oracle sweep (the strategies of tests/test_properties.py, not
derandomized): python tools/fuzz_gpu.py [--examples 2000] [--seed S] [--which configs,csr,binned,partitions,resume,steps,hubs,dense]

Prints one line per strategy with the number of passing draws, or the falsifying example.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "approximate-consensus-simulation_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--examples", type=int, default=2000)
    ap.add_argument("--seed", type=int, default=12345)
    ap.add_argument("--which", default="configs,csr,binned,partitions,resume,steps")
    a = ap.parse_args()
    from hypothesis import HealthCheck, given, seed, settings
    import oracle
    import test_properties as T
    oracle.build()
    tests = {
        "configs": (T.test_gpu_matches_oracle_random_configs, "cfg", T.configs(max_n=400)),
        "csr": (T.test_gpu_matches_oracle_random_csr, "case", T.csr_configs(max_n=600)),
        "binned": (T.test_gpu_binned_exchange_random_configs, "case", T.binned_configs()),
        "partitions": (T.test_gpu_virtual_partitions_random_configs, "case", T.partition_cases()),
    }
    from hypothesis import strategies as st
    multi = {   # tests with two drawn arguments
        "resume": (T.test_gpu_resume_random_configs, {"cfg": T.configs(max_n=300), "frac": st.floats(0.0, 1.0)}),
        "steps": (T.test_gpu_round_steps_equal_run,
                  {"cfg": T.configs(max_n=300), "steps": st.lists(st.integers(1, 17), min_size=1, max_size=6)}),
    }
    for name, (fn, args) in multi.items():
        tests[name] = (fn, args, None)

    # CSR graphs with hub rows (fast path + generic size classes + the big-m path above 8192
    # entries): a few heavy draws, checked like test_gpu_matches_oracle_random_csr
    import numpy as np

    @st.composite
    def hub_cases(draw):
        n = draw(st.integers(9000, 20000))
        rng = np.random.default_rng(draw(st.integers(0, 2 ** 32)))
        deg = rng.integers(draw(st.integers(3, 11)), 33, size=n)
        nh = draw(st.integers(1, 6))
        hubs = rng.choice(n, size=nh, replace=False)
        deg[hubs] = rng.integers(40, 12000, size=nh)
        rowptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.uint64)
        colidx = rng.integers(0, n, size=int(rowptr[-1])).astype(np.uint32)
        base = draw(T.configs())
        tmax = int(deg.min()) // 2
        rule = base.rule
        t = 0 if rule == "average" else draw(st.integers(1 if rule == "dlpsw" else 0, max(tmax, 1)))
        if t > tmax:
            rule, t = "average", 0
        cfg = base.replace(topology="csr", n_nodes=n, degree=0, rule=rule, trim=t, n_instances=1,
                           n_faulty=min(base.n_faulty, n // 10), max_rounds=min(base.max_rounds, 12))
        return cfg, (rowptr, colidx)

    tests["hubs"] = (T.test_gpu_matches_oracle_random_csr, "case", hub_cases())

    # complete graphs the persistent dense kernel serves (asserts the kernel; up to 2048 nodes)
    tests["dense"] = (T.test_gpu_dense_random_configs, "cfg", T.dense_configs(max_n=2048))
    for name in a.which.split(","):
        if name not in tests:
            continue
        fn, arg, strat = tests[name]
        given_kw = arg if strat is None else {arg: strat}
        inner = fn.hypothesis.inner_test
        import inspect
        takes_oracle = "oracle_mod" in inspect.signature(inner).parameters
        n = [0]
        failing = []

        def body(**kw):
            n[0] += 1
            try:
                if takes_oracle:
                    inner(oracle, **kw)
                else:
                    inner(**kw)
            except Exception:
                failing.append(kw)   # the last one is hypothesis' shrunk example
                raise

        t0 = time.time()
        run = seed(a.seed)(settings(max_examples=a.examples, deadline=None, database=None,
                                    suppress_health_check=list(HealthCheck))(given(**given_kw)(body)))
        try:
            run()
            print(f"{name}: {n[0]} draws passed in {time.time() - t0:.0f} s", flush=True)
        except Exception as e:  # noqa: BLE001
            print(f"{name}: FAILED after {n[0]} draws: {type(e).__name__}: {e}", flush=True)
            if failing:
                print(f"  smallest failing example: {failing[-1]!r}", flush=True)


if __name__ == "__main__":
    main()
