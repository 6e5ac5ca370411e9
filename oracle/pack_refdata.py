"""ORACLE TEST INFRASTRUCTURE -- packs the reference's own CMBlikes data files
(data, not source) that the CMBlikes parity tests read into
tests/golden/refdata.tar.xz, so the tests run where /root/reference is absent
(the GPU box).  Files are copied verbatim from /root/reference/data:

  planck_calib.paramnames
  planck_lensing_2018/...consext8 (dataset, bandpowers, cov, fiducial correction, windows)
  BKPlanck/BKPlanck_detset_comb_* + BKPlanck.paramnames + the five used bandpasses + windows
  sptsz_2500d_tt/*
  BK15/* (all but the bandpower covariance, which the reference does not ship;
          cosmomc_amd.synthetic.write_bk15_covmat writes a synthetic one after extraction)

    python oracle/pack_refdata.py
"""
import io
import lzma
import os
import tarfile

REF = "/root/reference/data"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "refdata.tar.xz")
LENS = "planck_lensing_2018/smicadx12_Dec5_ftl_mv2_ndclpp_p_teb_consext8"


def members():
    yield "planck_calib.paramnames"
    for suf in (".dataset", "_bandpowers.dat", "_cov.dat", "_lensing_fiducial_correction.dat"):
        yield LENS + suf
    for d in ("_window", "_lens_delta_window"):
        for f in sorted(os.listdir(os.path.join(REF, LENS + d))):
            yield f"{LENS}{d}/{f}"
    for f in sorted(os.listdir(os.path.join(REF, "BKPlanck"))):
        if f.startswith("BKPlanck_detset_comb_") or f == "BKPlanck.paramnames":
            yield "BKPlanck/" + f
    for b in ("B2K", "P100", "P143", "P217", "P353"):
        yield f"BKPlanck/bandpass_{b}.txt"
    for f in sorted(os.listdir(os.path.join(REF, "BKPlanck", "windows"))):
        if f.startswith("BKPlanck_detset_comb_bpwf_bin"):
            yield "BKPlanck/windows/" + f
    for d in ("sptsz_2500d_tt", "BK15"):
        for root, _, files in sorted(os.walk(os.path.join(REF, d))):
            for f in sorted(files):
                yield os.path.relpath(os.path.join(root, f), REF)


def main():
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w") as tar:
        for m in members():
            info = tar.gettarinfo(os.path.join(REF, m), arcname=m)
            info.mtime, info.uid, info.gid, info.uname, info.gname, info.mode = 0, 0, 0, "", "", 0o644
            with open(os.path.join(REF, m), "rb") as f:
                tar.addfile(info, f)
    with open(OUT, "wb") as f:
        f.write(lzma.compress(buf.getvalue(), preset=9))
    print(OUT, os.path.getsize(OUT))


if __name__ == "__main__":
    main()
