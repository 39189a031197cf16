"""Round-4 PSNR-parity tables for DESIGN §8 (test infrastructure): merges the finished oracle
ensemble members of profiles/round4/ensemble_* into fixtures, runs tests/psnr_ensemble.py's paired
statistics and prints markdown rows.  Usage: python tools/psnr_round4_tables.py"""
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PE = os.path.join(ROOT, "tests", "psnr_ensemble.py")
R4 = os.path.join(ROOT, "profiles", "round4")


def finished(d):
    out = []
    for f in sorted(glob.glob(os.path.join(R4, d, "ref_member*.json")), key=lambda p: int(p.split("member")[-1][:-5])):
        r = json.load(open(f))
        if r.get("placeholder") or not r.get("curve") or r["curve"][-1]["step"] != r.get("steps"):
            continue
        out.append(f)
    return out


def merge(d, out):
    files = finished(d)
    subprocess.run([sys.executable, PE, "merge", *files, "--out", out], check=True, stdout=subprocess.DEVNULL)
    return len(files)


def compare(a, b, out=None):
    cmd = [sys.executable, PE, "compare", a, b] + (["--out", out] if out else [])
    res = subprocess.run(cmd, check=True, capture_output=True, text=True).stdout
    return [json.loads(l) for l in res.splitlines() if l.startswith("{")]


def rows(st, steps=(125, 250, 500, 750, 1000)):
    for s in st:
        if s["step"] in steps:
            ci = s["paired_delta_ci95"]
            print(f"| {s['step']} | {s['members']} | {s['oracle_mean']:.3f} ± {s['oracle_se']:.3f} | "
                  f"{s['hip_mean']:.3f} ± {s['hip_se']:.3f} | **{s['paired_delta_mean']:+.3f} ± {s['paired_delta_se']:.3f}** | "
                  f"[{ci[0]:+.2f}, {ci[1]:+.2f}] | {s['paired_delta_sd']:.3f} |")


if __name__ == "__main__":
    G = os.path.join(ROOT, "tests", "golden")
    n = merge("ensemble_f16bw_refsamp", os.path.join(G, "psnr_oracle_ensemble_f16bw_refsamp.json"))
    print(f"## reference-style grid sampling oracle ({n} members) vs device-sampling oracle (B)")
    rows(compare(os.path.join(G, "psnr_oracle_ensemble_f16bw_refsamp.json"), os.path.join(G, "psnr_oracle_ensemble_f16bw.json"),
                 os.path.join(R4, "psnr_refsamp_vs_f16bw_oracle.json")))
    print("## HIP vs reference-style grid sampling oracle")
    rows(compare(os.path.join(R4, "psnr_hip_ensemble.json"), os.path.join(G, "psnr_oracle_ensemble_f16bw_refsamp.json"),
                 os.path.join(R4, "psnr_hip_vs_f16bw_refsamp_oracle.json")))
    n = merge("ensemble_scannet_f16bw", os.path.join(G, "psnr_oracle_ensemble_scannet_f16bw.json"))
    print(f"## config #5: HIP vs fp16-fw+bw oracle ({n} members)")
    rows(compare(os.path.join(R4, "psnr_hip_ensemble_scannet.json"), os.path.join(G, "psnr_oracle_ensemble_scannet_f16bw.json"),
                 os.path.join(R4, "psnr_hip_vs_f16bw_oracle_scannet.json")))
    print("## config #5: fp16-fw+bw oracle vs fp32 oracle")
    rows(compare(os.path.join(G, "psnr_oracle_ensemble_scannet_f16bw.json"), os.path.join(G, "psnr_oracle_ensemble_scannet.json"),
                 os.path.join(R4, "psnr_f16bw_vs_fp32_oracle_scannet.json")))
