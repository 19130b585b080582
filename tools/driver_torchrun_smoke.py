#!/usr/bin/env python3
"""The N-GPU driver (python -m hakai.run under torch.distributed.run, --nproc ranks; on a one-GPU box
the ranks share the device and RCCL connects them over loopback, hakai.dist.rank_device; this
script sets HAKAI_RCCL_SHARED_GPU=1 for its ranks): writes a
contact deck with deletions, runs the one-GPU driver (hakai.hakai) and the torchrun driver, and
compares their VTK files byte for byte."""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hakai-fem_amd"), os.path.join(ROOT, "tests")]


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--nproc", type=int, default=2)
    args = ap.parse_args()
    import hakai
    from hakai import mesh
    from inp_writer import write_inp
    tmp = tempfile.mkdtemp(prefix="hakai_tr_")
    m = mesh.two_body_model(plate=(6, 6, 1), impactor=(2, 2, 3), v=-3e5, d_time=2e-8, n_steps=400)
    deck = write_inp(os.path.join(tmp, "impact.inp"), m)
    hakai.hakai(deck, os.path.join(tmp, "one"), verbose=False)
    env = dict(os.environ, HAKAI_RCCL_SHARED_GPU="1", PYTHONPATH=os.path.join(ROOT, "hakai-fem_amd") + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.nproc),
                        "--master-addr", "127.0.0.1", "--master-port", "29561", "-m", "hakai.run", deck,
                        os.path.join(tmp, "multi")], env=env, capture_output=True, text=True, timeout=300)
    print(r.stdout[-2000:], r.stderr[-2000:])
    if r.returncode:
        return r.returncode
    a, b = sorted(os.listdir(os.path.join(tmp, "one"))), sorted(os.listdir(os.path.join(tmp, "multi")))
    same = a == b and all(open(os.path.join(tmp, "one", f), "rb").read() == open(os.path.join(tmp, "multi", f), "rb").read()
                          for f in a)
    print(f"torchrun driver (world {args.nproc}) vs one-GPU driver: {len(a)} files, byte-identical: {same}")
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main())
