"""Factor error of the albedo protocol fit (tests/test_gpu_heavy_tail.py::
test_albedo_protocol_at_c1_hyperparameters) against the fp64 oracle, for the library named by
ALBEDO_ALS_LIB; run twice to check run-to-run identity.  Diagnostic, GPU box only.
usage: python tools/protocol_eu.py <tag>"""
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from oracle import spark_als as O  # noqa: E402
from albedo_amd import ALSModel, builder  # noqa: E402


def _rel(a, b):
    return float(np.max(np.abs(a - b)) / np.max(np.abs(b)))


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "lib"
    users, repos, stars_n = 3000, 800, 40000
    stars = builder.load_raw_starring(users, repos, stars_n, 42)
    B = O.make_blocks(stars["user_id"], stars["repo_id"], stars["starring"].astype(np.float32))
    su, si = O.spark_side_seeds(42)
    U, V = O.fit(B, rank=50, max_iter=26, reg=0.5, alpha=40.0, init_user=O.spark_initialize(B.user_ids, 50, su),
                 init_item=O.spark_initialize(B.item_ids, 50, si))
    prev = None
    for rep in range(2):
        with tempfile.TemporaryDirectory() as td:
            path = os.path.join(td, "m.parquet")
            builder.main(["--users", str(users), "--repos", str(repos), "--stars", str(stars_n), "--rank", "50",
                          "--max-iter", "26", "--top-k", "30", "--model-path", path])
            m = ALSModel.load(path)
            uf, itf = m.user_factors_np()[1], m.item_factors_np()[1]
        same = prev is not None and np.array_equal(prev[0], uf) and np.array_equal(prev[1], itf)
        print(f"{tag} rep {rep}: eu {_rel(uf, U):.3e} ev {_rel(itf, V):.3e} identical_to_prev {same}", flush=True)
        prev = (uf, itf)


if __name__ == "__main__":
    main()
