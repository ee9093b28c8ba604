"""Build the in-tree artefacts: libtachyon_mi355x.so (hipcc, gfx950) and the
oracle's liboracle.so (gcc; test infrastructure only)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def build_library(jobs: int = 8):
    subprocess.run(["make", "-s", f"-j{jobs}", "-C", os.path.join(ROOT, "tachyon_amd", "csrc")], check=True)


def build_oracle():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)


if __name__ == "__main__":
    build_library()
    build_oracle()
