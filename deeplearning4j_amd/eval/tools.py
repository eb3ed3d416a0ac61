"""EvaluationTools: standalone HTML reports of ROC / precision-recall curves and calibration charts (reference
deeplearning4j-core/src/main/java/org/deeplearning4j/evaluation/EvaluationTools.java:106-230).

The reference renders through its UI component library and FreeMarker templates; here every chart is inline SVG in
one self-contained HTML page (no scripts, no external assets), so reports open offline and can be attached to CI
artifacts. Text is HTML-escaped."""
import html

import numpy as np

_W, _H, _PAD = 480, 320, 44


def _fmt(v):
    return f"{v:.4g}"


def _line_chart(title, xs_list, ys_list, names, xlabel, ylabel, xr=(0.0, 1.0), yr=(0.0, 1.0), diagonal=False):
    """One SVG line chart; each (xs, ys) pair is a series."""
    x0, x1 = xr
    y0, y1 = yr
    sx = lambda x: _PAD + (x - x0) / max(x1 - x0, 1e-12) * (_W - 2 * _PAD)      # noqa: E731
    sy = lambda y: _H - _PAD - (y - y0) / max(y1 - y0, 1e-12) * (_H - 2 * _PAD)  # noqa: E731
    colors = ["#1f77b4", "#d62728", "#2ca02c", "#9467bd", "#ff7f0e", "#8c564b", "#e377c2", "#17becf"]
    out = [f'<svg xmlns="http://www.w3.org/2000/svg" width="{_W}" height="{_H}" class="chart">',
           f'<text x="{_W / 2}" y="16" text-anchor="middle" font-weight="bold">{html.escape(title)}</text>',
           f'<rect x="{_PAD}" y="{_PAD}" width="{_W - 2 * _PAD}" height="{_H - 2 * _PAD}" fill="none" stroke="#999"/>']
    for t in np.linspace(0, 1, 6):
        xv, yv = x0 + t * (x1 - x0), y0 + t * (y1 - y0)
        out.append(f'<text x="{sx(xv):.1f}" y="{_H - _PAD + 14}" text-anchor="middle" font-size="10">{_fmt(xv)}</text>')
        out.append(f'<text x="{_PAD - 4}" y="{sy(yv) + 3:.1f}" text-anchor="end" font-size="10">{_fmt(yv)}</text>')
    out.append(f'<text x="{_W / 2}" y="{_H - 8}" text-anchor="middle" font-size="11">{html.escape(xlabel)}</text>')
    out.append(f'<text x="12" y="{_H / 2}" text-anchor="middle" font-size="11" '
               f'transform="rotate(-90 12 {_H / 2})">{html.escape(ylabel)}</text>')
    if diagonal:
        out.append(f'<line x1="{sx(x0):.1f}" y1="{sy(y0):.1f}" x2="{sx(x1):.1f}" y2="{sy(y1):.1f}" '
                   f'stroke="#bbb" stroke-dasharray="4 3"/>')
    for k, (xs, ys) in enumerate(zip(xs_list, ys_list)):
        pts = " ".join(f"{sx(float(x)):.1f},{sy(float(y)):.1f}" for x, y in zip(xs, ys)
                       if np.isfinite(x) and np.isfinite(y))
        c = colors[k % len(colors)]
        out.append(f'<polyline fill="none" stroke="{c}" stroke-width="1.5" points="{pts}"/>')
        if names and len(xs_list) > 1:
            out.append(f'<text x="{_W - _PAD - 4}" y="{_PAD + 14 + 13 * k}" text-anchor="end" font-size="10" '
                       f'fill="{c}">{html.escape(str(names[k]))}</text>')
    out.append("</svg>")
    return "".join(out)


def _histogram(hist):
    counts = np.asarray(hist.binCounts, dtype=np.float64)
    n = len(counts)
    top = max(1.0, float(counts.max()) if n else 1.0)
    bw = (_W - 2 * _PAD) / max(n, 1)
    out = [f'<svg xmlns="http://www.w3.org/2000/svg" width="{_W}" height="{_H}" class="chart">',
           f'<text x="{_W / 2}" y="16" text-anchor="middle" font-weight="bold">{html.escape(hist.title)}</text>',
           f'<rect x="{_PAD}" y="{_PAD}" width="{_W - 2 * _PAD}" height="{_H - 2 * _PAD}" fill="none" stroke="#999"/>']
    for i, c in enumerate(counts):
        h = c / top * (_H - 2 * _PAD)
        out.append(f'<rect x="{_PAD + i * bw:.1f}" y="{_H - _PAD - h:.1f}" width="{max(bw - 1, 0.5):.1f}" '
                   f'height="{h:.1f}" fill="#1f77b4"><title>{int(c)}</title></rect>')
    out.append(f'<text x="{_PAD}" y="{_H - _PAD + 14}" font-size="10">{_fmt(hist.lower)}</text>')
    out.append(f'<text x="{_W - _PAD}" y="{_H - _PAD + 14}" text-anchor="end" font-size="10">{_fmt(hist.upper)}</text>')
    out.append(f'<text x="{_PAD - 4}" y="{_PAD + 4}" text-anchor="end" font-size="10">{int(top)}</text>')
    out.append("</svg>")
    return "".join(out)


def _page(title, sections):
    body = "".join(f"<h2>{html.escape(h)}</h2><div>{''.join(charts)}</div>" for h, charts in sections)
    return ("<!DOCTYPE html><html><head><meta charset=\"utf-8\"><title>" + html.escape(title) + "</title>"
            "<style>body{font-family:sans-serif;margin:20px}svg.chart{margin:6px;background:#fff}"
            "table{border-collapse:collapse}td,th{border:1px solid #ccc;padding:2px 8px}</style></head><body>"
            f"<h1>{html.escape(title)}</h1>{body}</body></html>")


def _roc_section(name, roc_curve, pr_curve, auc, aucpr):
    roc = _line_chart(f"ROC - {name} (AUC={auc:.4f})", [roc_curve.fpr], [roc_curve.tpr], None,
                      "False Positive Rate", "True Positive Rate", diagonal=True)
    pr = _line_chart(f"Precision-Recall - {name} (AUPRC={aucpr:.4f})", [pr_curve.recall], [pr_curve.precision],
                     None, "Recall", "Precision")
    return name, [roc, pr]


class EvaluationTools:
    """Static HTML exporters with the reference's names."""

    @staticmethod
    def rocChartToHtml(roc, classNames=None):
        from .roc import ROC, ROCBinary, ROCMultiClass
        if isinstance(roc, ROC):
            return _page("ROC", [_roc_section("ROC", roc.getRocCurve(), roc.getPrecisionRecallCurve(),
                                              roc.calculateAUC(), roc.calculateAUCPR())])
        if isinstance(roc, (ROCMultiClass, ROCBinary)):
            n = roc.getNumClasses() if isinstance(roc, ROCMultiClass) else roc.numLabels()
            if classNames is not None and len(classNames) != n:
                raise ValueError(f"{len(classNames)} class names for {n} classes")
            names = list(classNames) if classNames is not None else [f"class {i}" for i in range(n)]
            secs = [_roc_section(names[i], roc.getRocCurve(i), roc.getPrecisionRecallCurve(i), roc.calculateAUC(i),
                                 roc.calculateAUCPR(i)) for i in range(n)]
            return _page("ROC (per class)", secs)
        raise TypeError(f"rocChartToHtml: unsupported evaluation {type(roc).__name__}")

    @staticmethod
    def exportRocChartsToHtmlFile(roc, file, classNames=None):
        with open(file, "w", encoding="utf-8") as f:
            f.write(EvaluationTools.rocChartToHtml(roc, classNames))

    @staticmethod
    def evaluationCalibrationToHtml(ec):
        n = ec.numClasses()
        if n <= 0:
            raise ValueError("evaluationCalibrationToHtml: the EvaluationCalibration has seen no data")
        rel = [ec.getReliabilityDiagram(i) for i in range(n)]
        rel_chart = _line_chart("Reliability diagram", [r.meanPredictedValueX for r in rel],
                                [r.fractionPositivesY for r in rel], [f"class {i}" for i in range(n)],
                                "Mean predicted value", "Fraction of positives", diagonal=True)
        counts = ("<table><tr><th>class</th><th>label count</th><th>prediction count</th></tr>"
                  + "".join(f"<tr><td>{i}</td><td>{int(a)}</td><td>{int(b)}</td></tr>"
                            for i, (a, b) in enumerate(zip(ec.getLabelCountsEachClass(),
                                                           ec.getPredictionCountsEachClass()))) + "</table>")
        resid = [_histogram(ec.getResidualPlotAllClasses())] + [_histogram(ec.getResidualPlot(i)) for i in range(n)]
        prob = [_histogram(ec.getProbabilityHistogramAllClasses())] + \
            [_histogram(ec.getProbabilityHistogram(i)) for i in range(n)]
        return _page("Evaluation calibration", [("Reliability", [rel_chart]), ("Counts", [counts]),
                                                ("Residuals |label - p|", resid), ("Probabilities", prob)])

    @staticmethod
    def exportevaluationCalibrationToHtmlFile(ec, file):
        with open(file, "w", encoding="utf-8") as f:
            f.write(EvaluationTools.evaluationCalibrationToHtml(ec))


rocChartToHtml = EvaluationTools.rocChartToHtml
exportRocChartsToHtmlFile = EvaluationTools.exportRocChartsToHtmlFile
evaluationCalibrationToHtml = EvaluationTools.evaluationCalibrationToHtml
exportevaluationCalibrationToHtmlFile = EvaluationTools.exportevaluationCalibrationToHtmlFile
