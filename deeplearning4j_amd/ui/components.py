"""UI components and static HTML rendering.

Reference: deeplearning4j-ui-components (components/chart: ChartLine, ChartScatter, ChartHistogram,
ChartHorizontalBar, ChartStackedArea, ChartTimeline; components/table ComponentTable; components/text ComponentText;
components/component ComponentDiv; components/decorator DecoratorAccordion; standalone/StaticPageUtil.renderHTML) —
used for offline reports such as training-stats timelines. Components serialise to JSON (``toJson``) and render to
self-contained HTML with inline SVG (no scripts or external assets).
"""
import html
import json


class Style:
    def __init__(self, width=600, height=300, **kw):
        self.width, self.height = width, height
        self.extra = kw

    def to_dict(self):
        return {"width": self.width, "height": self.height, **self.extra}


StyleChart = StyleTable = StyleText = StyleDiv = Style

_COLORS = ["#1f77b4", "#ff7f0e", "#2ca02c", "#d62728", "#9467bd", "#8c564b", "#e377c2", "#7f7f7f"]


class Component:
    TYPE = "Component"

    def __init__(self, title=None, style=None):
        self.title = title
        self.style = style or Style()

    def to_dict(self):
        return {"componentType": self.TYPE, "title": self.title, "style": self.style.to_dict()}

    def toJson(self):
        return json.dumps(self.to_dict())

    def render(self):
        raise NotImplementedError

    def _frame(self, body):
        t = f"<h4>{html.escape(self.title)}</h4>" if self.title else ""
        return f'<div class="dl4j-component">{t}{body}</div>'


class _Chart(Component):
    def __init__(self, title=None, style=None):
        super().__init__(title, style)
        self.series = []            # (name, xs, ys)

    def addSeries(self, name, x, y):
        self.series.append((name, [float(v) for v in x], [float(v) for v in y]))
        return self

    def to_dict(self):
        d = super().to_dict()
        d["series"] = [{"name": n, "x": x, "y": y} for n, x, y in self.series]
        return d

    def _bounds(self):
        xs = [v for _, x, _ in self.series for v in x] or [0, 1]
        ys = [v for _, _, y in self.series for v in y] or [0, 1]
        x0, x1, y0, y1 = min(xs), max(xs), min(ys), max(ys)
        return x0, (x1 if x1 > x0 else x0 + 1), y0, (y1 if y1 > y0 else y0 + 1)

    def _svg(self, marks):
        w, h = self.style.width, self.style.height
        x0, x1, y0, y1 = self._bounds()
        sx = lambda v: 40 + (v - x0) / (x1 - x0) * (w - 50)  # noqa: E731
        sy = lambda v: h - 20 - (v - y0) / (y1 - y0) * (h - 30)  # noqa: E731
        body = "".join(marks(i, x, y, sx, sy) for i, (_, x, y) in enumerate(self.series))
        legend = "".join(f'<text x="{w - 120}" y="{14 + 12 * i}" font-size="10" fill="{_COLORS[i % 8]}">'
                         f"{html.escape(n)}</text>" for i, (n, _, _) in enumerate(self.series))
        axes = (f'<text x="2" y="12" font-size="10">{y1:.4g}</text><text x="2" y="{h - 22}" font-size="10">'
                f'{y0:.4g}</text><text x="40" y="{h - 4}" font-size="10">{x0:.4g}</text>'
                f'<text x="{w - 40}" y="{h - 4}" font-size="10">{x1:.4g}</text>')
        return f'<svg width="{w}" height="{h}" style="background:#fff">{body}{legend}{axes}</svg>'


class ChartLine(_Chart):
    TYPE = "ChartLine"

    def render(self):
        def marks(i, x, y, sx, sy):
            pts = " ".join(f"{sx(a):.1f},{sy(b):.1f}" for a, b in zip(x, y))
            return f'<polyline fill="none" stroke="{_COLORS[i % 8]}" points="{pts}"/>'
        return self._frame(self._svg(marks))


class ChartScatter(_Chart):
    TYPE = "ChartScatter"

    def render(self):
        def marks(i, x, y, sx, sy):
            return "".join(f'<circle cx="{sx(a):.1f}" cy="{sy(b):.1f}" r="2" fill="{_COLORS[i % 8]}"/>'
                           for a, b in zip(x, y))
        return self._frame(self._svg(marks))


class ChartStackedArea(_Chart):
    TYPE = "ChartStackedArea"

    def render(self):
        if self.series:
            acc = [0.0] * len(self.series[0][1])
            stacked = []
            for n, x, y in self.series:
                acc = [a + b for a, b in zip(acc, y)]
                stacked.append((n, x, list(acc)))
            self.series = stacked

        def marks(i, x, y, sx, sy):
            pts = " ".join(f"{sx(a):.1f},{sy(b):.1f}" for a, b in zip(x, y))
            return f'<polyline fill="none" stroke="{_COLORS[i % 8]}" stroke-width="2" points="{pts}"/>'
        return self._frame(self._svg(marks))


class ChartHistogram(Component):
    TYPE = "ChartHistogram"

    def __init__(self, title=None, style=None):
        super().__init__(title, style)
        self.bins = []               # (lower, upper, y)

    def addBin(self, lower, upper, y):
        self.bins.append((float(lower), float(upper), float(y)))
        return self

    def to_dict(self):
        d = super().to_dict()
        d["bins"] = [{"lower": a, "upper": b, "y": y} for a, b, y in self.bins]
        return d

    def render(self):
        w, h = self.style.width, self.style.height
        if not self.bins:
            return self._frame("(empty)")
        lo, hi = min(b[0] for b in self.bins), max(b[1] for b in self.bins)
        ym = max(b[2] for b in self.bins) or 1.0
        rects = "".join(
            f'<rect x="{40 + (a - lo) / ((hi - lo) or 1) * (w - 50):.1f}" y="{h - 20 - y / ym * (h - 30):.1f}" '
            f'width="{max(1.0, (b - a) / ((hi - lo) or 1) * (w - 50)):.1f}" height="{y / ym * (h - 30):.1f}" '
            f'fill="#1f77b4"/>' for a, b, y in self.bins)
        return self._frame(f'<svg width="{w}" height="{h}" style="background:#fff">{rects}</svg>')


class ChartHorizontalBar(Component):
    TYPE = "ChartHorizontalBar"

    def __init__(self, title=None, style=None):
        super().__init__(title, style)
        self.labels, self.values = [], []

    def addValue(self, label, value):
        self.labels.append(str(label))
        self.values.append(float(value))
        return self

    def to_dict(self):
        d = super().to_dict()
        d["labels"], d["values"] = self.labels, self.values
        return d

    def render(self):
        w = self.style.width
        vm = max([abs(v) for v in self.values] + [1e-30])
        bh = 16
        rows = "".join(f'<text x="0" y="{i * bh + 12}" font-size="10">{html.escape(l)}</text>'
                       f'<rect x="120" y="{i * bh + 2}" width="{abs(v) / vm * (w - 130):.1f}" height="{bh - 4}" '
                       f'fill="#2ca02c"/>' for i, (l, v) in enumerate(zip(self.labels, self.values)))
        return self._frame(f'<svg width="{w}" height="{len(self.values) * bh + 4}">{rows}</svg>')


class ChartTimeline(Component):
    TYPE = "ChartTimeline"

    def __init__(self, title=None, style=None):
        super().__init__(title, style)
        self.lanes = []              # (laneName, [(start, end, label)])

    def addLaneData(self, name, entries):
        self.lanes.append((name, [(float(a), float(b), str(l)) for a, b, l in entries]))
        return self

    def to_dict(self):
        d = super().to_dict()
        d["lanes"] = [{"name": n, "entries": e} for n, e in self.lanes]
        return d

    def render(self):
        w = self.style.width
        all_t = [t for _, es in self.lanes for a, b, _ in es for t in (a, b)] or [0, 1]
        t0, t1 = min(all_t), max(all_t)
        span = (t1 - t0) or 1.0
        lh = 20
        out = []
        for i, (n, es) in enumerate(self.lanes):
            out.append(f'<text x="0" y="{i * lh + 14}" font-size="10">{html.escape(n)}</text>')
            for k, (a, b, l) in enumerate(es):
                out.append(f'<rect x="{100 + (a - t0) / span * (w - 110):.1f}" y="{i * lh + 3}" '
                           f'width="{max(1.0, (b - a) / span * (w - 110)):.1f}" height="{lh - 6}" '
                           f'fill="{_COLORS[k % 8]}"><title>{html.escape(l)}</title></rect>')
        return self._frame(f'<svg width="{w}" height="{len(self.lanes) * lh + 4}">{"".join(out)}</svg>')


class ComponentTable(Component):
    TYPE = "ComponentTable"

    def __init__(self, header=None, content=None, title=None, style=None):
        super().__init__(title, style)
        self.header = list(header or [])
        self.content = [list(r) for r in (content or [])]

    def to_dict(self):
        d = super().to_dict()
        d["header"], d["content"] = self.header, self.content
        return d

    def render(self):
        h = "".join(f"<th>{html.escape(str(c))}</th>" for c in self.header)
        rows = "".join("<tr>" + "".join(f"<td>{html.escape(str(c))}</td>" for c in r) + "</tr>" for r in self.content)
        return self._frame(f'<table border="1" cellpadding="3"><tr>{h}</tr>{rows}</table>')


class ComponentText(Component):
    TYPE = "ComponentText"

    def __init__(self, text="", title=None, style=None):
        super().__init__(title, style)
        self.text = text

    def to_dict(self):
        d = super().to_dict()
        d["text"] = self.text
        return d

    def render(self):
        return self._frame(f"<p>{html.escape(self.text)}</p>")


class ComponentDiv(Component):
    TYPE = "ComponentDiv"

    def __init__(self, *children, style=None):
        super().__init__(None, style)
        self.children = list(children)

    def to_dict(self):
        d = super().to_dict()
        d["components"] = [c.to_dict() for c in self.children]
        return d

    def render(self):
        return "<div>" + "".join(c.render() for c in self.children) + "</div>"


class DecoratorAccordion(ComponentDiv):
    TYPE = "DecoratorAccordion"

    def __init__(self, title, *children, defaultCollapsed=False):
        super().__init__(*children)
        self.title = title
        self.collapsed = defaultCollapsed

    def render(self):
        open_ = "" if self.collapsed else " open"
        return (f"<details{open_}><summary>{html.escape(self.title or '')}</summary>" +
                "".join(c.render() for c in self.children) + "</details>")


class StaticPageUtil:
    @staticmethod
    def renderHTML(*components):
        comps = components[0] if len(components) == 1 and isinstance(components[0], (list, tuple)) else components
        body = "".join(c.render() for c in comps)
        return ("<!doctype html><html><head><meta charset='utf-8'><title>DL4J-AMD report</title><style>"
                "body{font-family:sans-serif;margin:16px}.dl4j-component{margin:12px 0}</style></head><body>"
                + body + "</body></html>")

    @staticmethod
    def saveHTMLFile(path, *components):
        with open(path, "w", encoding="utf-8") as fh:
            fh.write(StaticPageUtil.renderHTML(*components))
