"""Copy a rocprofv3 --stats kernel summary into profiles/ with the build it describes.
    python tools/prof_record.py <rocprof -d dir> <profiles/r05_vN_<mode>_kernel_stats.csv> "<command>"
Writes the csv and <same name>.meta.json = {lib_sha256, git_head (CLIMSR_GIT_HEAD), command}: the library hash is
what bench.py / the judge match against the benched build."""
import glob
import hashlib
import json
import os
import shutil
import sys

LIB = os.environ.get("CLIMSR_HIP_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                     "climate-super-resolution_amd", "csrc", "libclimsr_hip.so"))


def main():
    src_dir, dst, cmd = sys.argv[1:4]
    files = glob.glob(os.path.join(src_dir, "**", "*kernel_stats.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no kernel_stats.csv under {src_dir}")
    shutil.copy(sorted(files)[-1], dst)
    meta = {"lib_sha256": hashlib.sha256(open(LIB, "rb").read()).hexdigest(), "git_head": os.environ.get("CLIMSR_GIT_HEAD"),
            "command": cmd}
    json.dump(meta, open(os.path.splitext(dst)[0] + ".meta.json", "w"), indent=1)
    print(dst, meta["lib_sha256"][:16])


if __name__ == "__main__":
    main()
