"""Recover the plotted closed-loop data of the reference's only acados-produced artefacts.

    python tests/golden/extract_reference_plots.py      (needs /root/reference; run here only)

`experiment_data/img/example_{acc,jerk}_*.pdf` are the matplotlib (PDF-1.4, Flate) plots of one
seed-42 `src/main.py` run (`main.py:43-46`): `acc` = force model (create_plots with a=None,
`main.py:26-28`), `jerk` = jerk model (`main.py:38-40`). The plotting code is
`src/store_results.py:21-230`. This script reads the PDF bytes as DATA: stdlib `zlib`
inflates the page content stream, the path operators (`x y m`, `x y l`, `S`) give the
polyline vertices in points, and the tick marks (3.5-pt segments on the axes edge) with their
text labels give each axis' affine map from points back to data units. Nothing from the
reference is imported or executed.

Output `tests/golden/reference_plots.npz`, per figure `<fig>` and data path `j`:
  `<fig>__p<j>`       vertices in data coordinates, (n, 2)
  `<fig>__p<j>_meta`  [axes index, colour code, dashed]  (colour code: 1 skyblue, 2 deepskyblue,
                      3 darkgreen — store_results.py:142-146 / :24-28)
  `<fig>__axes`       per axes [x0, x1, y0, y1] of the clip box in points and the fitted maps
                      [ax, bx, ay, by]: data = a * points + b
The component figures (`*_trajectory_component`) plot against time x = arange(0, T, dt)
(`store_results.py:151`), so every surviving vertex there is one sample: index = t / dt.
Matplotlib path simplification drops near-collinear vertices but keeps the ones it writes.
"""
import os
import re
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
IMG = "/root/reference/experiment_data/img"
FIGS = ["example_acc_traj_pos", "example_acc_traj_vel", "example_acc_trajectory_component",
        "example_jerk_traj_pos", "example_jerk_traj_vel", "example_jerk_traj_acc",
        "example_jerk_trajectory_component"]
COLOURS = {(0.5294117647, 0.8078431373, 0.9215686275): 1,   # skyblue
           (0.0, 0.7490196078, 1.0): 2,                     # deepskyblue
           (0.0, 0.3921568627, 0.0): 3}                     # darkgreen


def content_stream(path):
    raw = open(path, "rb").read()
    cid = re.search(rb"/Contents (\d+) 0 R", raw).group(1)
    m = re.search(rb"\n" + cid + rb" 0 obj.*?stream\r?\n(.*?)\r?\nendstream", raw, re.S)
    return zlib.decompress(m.group(1)).decode("latin1")


def tokens(s):
    """PDF content tokens: numbers, names, operators, (strings), [arrays] kept whole."""
    return re.findall(r"\((?:\\.|[^\\)])*\)|\[[^\]]*\]|/[^\s/\[\]()]+|[^\s\[\]()/]+", s)


def label_text(chunks):
    """Tick label glyphs -> text. F1 is CMSY10 (code 0 = minus), F3 CMMI12 (':' is the
    period glyph), F2/F4 CMR digits."""
    out = ""
    for font, txt in chunks:
        for ch in txt:
            if font == "/F1" and ch == "\x00":
                out += "-"
            elif font == "/F3" and ch == ":":
                out += "."
            else:
                out += ch
    return out


def parse(path):
    s = content_stream(path)
    tk = tokens(s)
    stack = []
    clip = None
    stroke = (0.0, 0.0, 0.0)
    dashed = False
    cur = []
    axes = []          # clip boxes in order of first appearance
    paths = []         # (axes idx, colour, dashed, pts)
    ticks = []         # (axes idx, 'x'|'y', position, label or None)
    pending_tick = None
    in_text = False
    font = None
    text = []

    def axis_of(box):
        for i, b in enumerate(axes):
            if np.allclose(b, box):
                return i
        axes.append(box)
        return len(axes) - 1

    for t in tk:
        if t == "BT":
            in_text, text = True, []
            continue
        if t == "ET":
            in_text = False
            if pending_tick is not None:
                lab = label_text(text)
                try:
                    val = float(lab.replace("−", "-"))
                except ValueError:
                    val = None
                a, kind, pos = pending_tick
                if val is not None:
                    ticks.append((a, kind, pos, val))
                pending_tick = None
            continue
        if in_text:
            if t == "Tf":
                font = stack[-2]
            elif t == "Tj":
                text.append((font, stack[-1][1:-1].replace("\\(", "(").replace("\\)", ")")))
            elif t == "TJ":
                for part in re.findall(r"\((?:\\.|[^\\)])*\)", stack[-1]):
                    text.append((font, part[1:-1]))
            if t in ("Tf", "Tj", "TJ", "Td"):
                stack = []
            else:
                stack.append(t)
            continue
        if t == "re":
            box = [float(v) for v in stack[-4:]]
            stack = []
            clip_pending = box
            continue
        if t == "W":
            clip = axis_of(clip_pending)
            stack = []
            continue
        if t == "Q":
            clip = None
            dashed = False
            stack = []
            continue
        if t == "RG":
            stroke = tuple(float(v) for v in stack[-3:])
            stack = []
            continue
        if t == "G":
            stroke = (float(stack[-1]),) * 3
            stack = []
            continue
        if t == "d":
            dashed = stack[-2] not in ("[ ]", "[]")
            stack = []
            continue
        if t == "m":
            cur = [(float(stack[-2]), float(stack[-1]))]
            stack = []
            continue
        if t == "l":
            cur.append((float(stack[-2]), float(stack[-1])))
            stack = []
            continue
        if t in ("S", "B"):
            pts = np.array(cur)
            if t == "B" and clip is None and len(pts) == 2 and axes:
                # tick mark: a 3.5-pt segment leaving the edge of the last axes box
                dx, dy = pts[1] - pts[0]
                if abs(dx) < 1e-9 and abs(abs(dy) - 3.5) < 1e-6:
                    a = _edge_axes(axes, pts[0], "x")
                    pending_tick = (a, "x", pts[0][0]) if a is not None else None
                elif abs(dy) < 1e-9 and abs(abs(dx) - 3.5) < 1e-6:
                    a = _edge_axes(axes, pts[0], "y")
                    pending_tick = (a, "y", pts[0][1]) if a is not None else None
            elif t == "S" and clip is not None and len(pts) > 8:
                col = next((c for k, c in COLOURS.items() if np.allclose(k, stroke, atol=1e-6)), 0)
                if col:
                    paths.append((clip, col, dashed, pts))
            cur = []
            stack = []
            continue
        stack.append(t)
    return axes, paths, ticks


def _edge_axes(axes, p, kind):
    for i, (x0, y0, w, h) in enumerate(axes):
        if kind == "x" and abs(p[1] - y0) < 1e-4 and x0 - 1e-4 <= p[0] <= x0 + w + 1e-4:
            return i
        if kind == "y" and abs(p[0] - x0) < 1e-4 and y0 - 1e-4 <= p[1] <= y0 + h + 1e-4:
            return i
    return None


def fit(pairs):
    px = np.array([q[0] for q in pairs])
    v = np.array([q[1] for q in pairs])
    A = np.vstack([px, np.ones_like(px)]).T
    (a, b), res, *_ = np.linalg.lstsq(A, v, rcond=None)
    resid = np.abs(A @ [a, b] - v).max()
    assert resid < 1e-6 * max(1.0, np.abs(v).max()), resid
    return a, b


def main():
    out = {}
    for fig in FIGS:
        axes, paths, ticks = parse(os.path.join(IMG, fig + ".pdf"))
        maps = []
        xticks_all = [(p, v) for a, k, p, v in ticks if k == "x"]
        for i in range(len(axes)):
            xt = [(p, v) for a, k, p, v in ticks if k == "x" and a == i] or xticks_all   # sharex
            yt = [(p, v) for a, k, p, v in ticks if k == "y" and a == i]
            if len(xt) < 2 or len(yt) < 2:
                maps.append([np.nan] * 4)
                continue
            ax_, bx_ = fit(xt)
            ay_, by_ = fit(yt)
            maps.append([ax_, bx_, ay_, by_])
        maps = np.array(maps)
        box = np.array(axes)
        out[f"{fig}__axes"] = np.hstack([box, maps])
        for j, (a, col, dashed, pts) in enumerate(paths):
            m = maps[a]
            data = np.stack([m[0] * pts[:, 0] + m[1], m[2] * pts[:, 1] + m[3]], axis=1)
            out[f"{fig}__p{j}"] = data
            out[f"{fig}__p{j}_meta"] = np.array([a, col, int(dashed)])
        print(fig, "axes", len(axes), "paths", [(a, c, d, len(p)) for a, c, d, p in paths])
    np.savez_compressed(os.path.join(HERE, "reference_plots.npz"), **out)
    print("wrote", os.path.join(HERE, "reference_plots.npz"))


if __name__ == "__main__":
    sys.exit(main())
