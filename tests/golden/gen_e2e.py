"""End-to-end golden for the citation driver, produced by the REFERENCE.

    python tests/golden/gen_e2e.py          # in the build container

Writes a learnable synthetic Planetoid dataset (tests/planetoid_synth.py, files
this repo creates) into a temporary directory, then
  * runs the reference's own citation.py there on CPU (--no-cuda, untuned) and
    records its printed validation/test accuracy;
  * imports the reference's load_citation + sgc_precompute on the same files
    and records SHA-256 of the propagated features (K = 2).
Output: tests/golden/e2e_citation.json.  The GPU test runs drivers/citation.py
on the same regenerated dataset and compares.
"""
import hashlib
import json
import os
import re
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("SGC_REFERENCE", "/root/reference")
sys.path.insert(0, os.path.join(ROOT, "tests"))

from planetoid_synth import write_planetoid  # noqa: E402

ARGS = ["--dataset", "synth", "--no-cuda", "--epochs", "100", "--degree", "2"]


def main():
    out = {}
    with tempfile.TemporaryDirectory() as d:
        spec = write_planetoid(d)
        env = dict(os.environ, PYTHONPATH=REF, PYTHONDONTWRITEBYTECODE="1")
        res = subprocess.run([sys.executable, os.path.join(REF, "citation.py"), *ARGS], cwd=d,
                             env=env, capture_output=True, text=True, check=True)
        m = re.search(r"Validation Accuracy: ([0-9.]+) Test Accuracy: ([0-9.]+)", res.stdout)
        out["reference_citation_py"] = {"args": ARGS, "val_acc": float(m.group(1)),
                                        "test_acc": float(m.group(2)), "stdout": res.stdout}
        code = (
            "import sys, hashlib, json; sys.path.insert(0, %r)\n"
            "import numpy as np\n"
            "from utils import load_citation, sgc_precompute\n"
            "adj, f, labels, itr, iva, ite = load_citation('synth', 'AugNormAdj', False)\n"
            "y, _ = sgc_precompute(f, adj, 2)\n"
            "h = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()\n"
            "print(json.dumps({'sha_adj_indices': h(adj._indices().numpy()),"
            " 'sha_adj_values': h(adj._values().numpy()), 'sha_features': h(f.numpy()),"
            " 'sha_precompute_K2': h(y.numpy()), 'n': int(f.shape[0])}))\n" % REF)
        res = subprocess.run([sys.executable, "-c", code], cwd=d, env=env, capture_output=True,
                             text=True, check=True)
        out["reference_load_and_precompute"] = json.loads(res.stdout.strip().splitlines()[-1])
        out["dataset"] = spec
    with open(os.path.join(HERE, "e2e_citation.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out["reference_citation_py"].items() if k != "stdout"}))


if __name__ == "__main__":
    main()
