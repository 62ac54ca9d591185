"""Digitise the min-voltage panel of the reference's single-component demo
notebook -- among the only OpenDSS power-flow outputs the reference holds
(examples/envs/multiagent-single-component.ipynb cell 6:
`df.min(axis=1).plot(title="min voltage", ...)` over env.history["voltage"],
one random-policy episode of three EV-charging agents on bus 675c, IEEE-13
through OpenDSSDirect.py) -- into tests/golden/notebook_minv.npz, the data of
tests/test_cpu_notebook_pin.py.

The two sibling notebooks (-multi-component, -heterogeneous) plot the same
panel, but their building agents' loads follow weather / PV series and
random thermostat actions whose range leaves an envelope tens of pixels wide:
no pin, so they are not digitised.

Runs in the build container only (it reads /root/reference; the fixture is
data: per 5-minute step the band of pu values the plotted line covers).  The
PNG is decoded here (zlib + PNG filters); the bottom panel's frame, its tick
marks and the line (matplotlib's C0 blue, antialiased) are found from the
pixels; the tick VALUES are read off the images by eye and written below.

Usage: python tools/digitize_notebook_plots.py
"""
import base64
import json
import os
import struct
import zlib

import numpy as np

REF = "/root/reference/examples/envs"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                   "notebook_minv.npz")
# notebook -> (scenario facts from its config cell, y tick labels of the min-voltage
# panel top to bottom, as printed in the image)
NOTEBOOKS = {
    "single": ("multiagent-single-component.ipynb", [0.97, 0.96, 0.95]),
}
X_TICK_HOURS = [3, 6, 9, 12, 15, 18, 21]          # "03:00" .. "21:00"
C0 = np.array([31, 119, 180])                       # matplotlib's default line colour


def read_png(data):
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, hdr = 8, b"", None
    while pos < len(data):
        n, typ = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        if typ == b"IHDR":
            hdr = struct.unpack(">IIBBBBB", body)
        elif typ == b"IDAT":
            idat += body
        pos += 12 + n
    w, h, depth, ctype, _, _, interlace = hdr
    assert depth == 8 and interlace == 0 and ctype in (2, 6), hdr
    ch = 3 if ctype == 2 else 4
    raw = np.frombuffer(zlib.decompress(idat), np.uint8)
    stride = w * ch
    out = np.zeros((h, stride), np.int32)
    prev = np.zeros(stride, np.int32)
    for y in range(h):
        f = raw[y * (stride + 1)]
        line = raw[y * (stride + 1) + 1:(y + 1) * (stride + 1)].astype(np.int32)
        if f == 0:
            cur = line.copy()
        elif f == 2:
            cur = (line + prev) & 255
        else:
            cur = np.zeros(stride, np.int32)
            for i in range(stride):
                a = cur[i - ch] if i >= ch else 0
                b = prev[i]
                c = prev[i - ch] if i >= ch else 0
                if f == 1:
                    v = a
                elif f == 3:
                    v = (a + b) // 2
                else:
                    pa, pb, pc = abs(b - c), abs(a - c), abs(a + b - 2 * c)
                    v = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
                cur[i] = (line[i] + v) & 255
        out[y] = cur
        prev = cur
    img = out.reshape(h, w, ch)
    if ch == 4:              # composite on white
        al = img[..., 3:4] / 255.0
        img = np.round(img[..., :3] * al + 255 * (1 - al)).astype(np.int32)
    return img


def panel(img):
    """(top, bottom, left, right) spine pixels of the bottom axes."""
    dark = img.sum(-1) < 200
    rows = np.nonzero(dark.sum(1) > 0.8 * dark.shape[1] * 0.85)[0]
    bottom = int(rows.max())
    top = int(rows[rows < bottom].max())
    cols = np.nonzero(dark[top + 2:bottom - 1].sum(0) >= (bottom - top - 3))[0]
    return top, bottom, int(cols.min()), int(cols.max())


def digitise(img, yvals):
    top, bottom, left, right = panel(img)
    grey = img.sum(-1) < 450                  # (tick marks are antialiased grey)
    # x ticks: marks under the bottom spine; y ticks: marks left of the left spine
    xt = np.nonzero(grey[bottom + 1, left + 1:right])[0] + left + 1
    yt = np.nonzero(grey[top + 1:bottom, left - 2] & grey[top + 1:bottom, left - 1])[0] + top + 1
    assert len(xt) == len(X_TICK_HOURS) and len(yt) == len(yvals), (xt, yt)
    ax, bx = np.polyfit(np.array(X_TICK_HOURS, float) * 60.0, xt.astype(float), 1)     # px = ax min + bx
    ay, by = np.polyfit(yt.astype(float), np.array(yvals), 1)                            # pu = ay row + by
    # the line: C0 blended with white (antialiasing): the pixel lies on the
    # segment white -> C0 within a few levels, with at least 25 % coverage
    sub = img[top + 1:bottom, left + 1:right].astype(float)
    t = (255.0 - sub) / (255.0 - C0)
    cov = t.mean(-1)
    resid = np.abs(sub - (255.0 - cov[..., None] * (255.0 - C0))).max(-1)
    line = (cov > 0.25) & (resid < 12)
    return dict(line=line, top=top, bottom=bottom, left=left, right=right, ax=ax, bx=bx, ay=ay, by=by)


def bands(d, minutes):
    """Per step (minutes since 00:00): the pu range the line covers within
    +-0.8 px of the step's x."""
    lo, hi = np.full(len(minutes), np.nan), np.full(len(minutes), np.nan)
    for k, m in enumerate(minutes):
        x = d["ax"] * m + d["bx"]
        c0, c1 = int(np.floor(x - 0.8)), int(np.ceil(x + 0.8))
        cols = [c - d["left"] - 1 for c in range(c0, c1 + 1) if d["left"] < c < d["right"]]
        rows = np.nonzero(d["line"][:, cols].any(1))[0] if cols else []
        if len(rows):
            r = rows + d["top"] + 1
            lo[k], hi[k] = d["ay"] * r.max() + d["by"], d["ay"] * r.min() + d["by"]
    return lo, hi


def main():
    out = {}
    for key, (nb, yvals) in NOTEBOOKS.items():
        cells = json.load(open(os.path.join(REF, nb)))["cells"]
        png = [base64.b64decode(o["data"]["image/png"]) for c in cells for o in c.get("outputs", [])
               if "data" in o and "image/png" in o["data"]]
        assert len(png) == 1
        d = digitise(read_png(png[0]), yvals)
        minutes = 5.0 * np.arange(1, 289)                     # the history's step times, 00:05 ..
        lo, hi = bands(d, minutes)
        keep = ~np.isnan(lo)
        out[key + "_minutes"] = minutes[keep]
        out[key + "_lo"], out[key + "_hi"] = lo[keep], hi[keep]
        out[key + "_pu_per_px"] = np.array(abs(d["ay"]))
        print(key, "frame", (d["top"], d["bottom"], d["left"], d["right"]), "steps", int(keep.sum()),
              "pu/px %.2e" % abs(d["ay"]), "range %.4f .. %.4f" % (np.nanmin(lo), np.nanmax(hi)))
    np.savez_compressed(OUT, **out)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
