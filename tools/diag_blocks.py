"""Block-kernel diagnostic (A/B builds): forces at C3 on sampled ions against the oracle, for each
value of the engine options given (MDQT_LIB selects the library build).
    MDQT_LIB=expt/<name>/lib/libmdqt.so python tools/diag_blocks.py NAME [opt=v,opt=v ...]"""
import os
import sys

ROOT = os.environ.get("MDQT_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402


def main(name, optsets):
    import mdqtplasmasims_amd as M
    from oracle import oracle as O
    s = M.Simulation(N0=100000, Ge=1.0 / 12, qt_enabled=0, seed=12346, job=1).init()
    R = s.get_state()["R"]
    idx = np.sort(np.random.default_rng(3).choice(s.N, 200, replace=False))
    idx = np.unique(np.concatenate([idx, np.arange(s.N - 64, s.N)]))
    G = O.forces_index(R, idx, s.const("L"), s.const("lDeb"), nthreads=16)
    for opts in optsets or [""]:
        for o in filter(None, opts.split(",")):
            k, v = o.split("=")
            s.set_option(k, int(v))
        s.forces()
        F = s.get_state()["F"]
        err = np.abs(F[:, idx] - G).max(axis=0) / np.abs(G).max()
        bad = idx[err > 1e-12]
        print(f"{name} [{opts}]: max rel err {err.max():.3e}; bad {len(bad)} of {len(idx)}: {bad[:12].tolist()}; "
              f"|F| sum {np.abs(F).sum():.6e}; zero rows {(np.abs(F).sum(axis=0) == 0).sum()}", flush=True)
    s.close()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
