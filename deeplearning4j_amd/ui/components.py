"""UI components and static HTML rendering.

Reference: deeplearning4j-ui-components (components/chart: ChartLine, ChartScatter, ChartHistogram,
ChartHorizontalBar, ChartStackedArea, ChartTimeline; components/table ComponentTable; components/text ComponentText;
components/component ComponentDiv; components/decorator DecoratorAccordion; standalone/StaticPageUtil.renderHTML) —
used for offline reports such as training-stats timelines. Components serialise to JSON (``toJson``) and render to
self-contained HTML with inline SVG (no scripts or external assets).
"""
import html
import json


class LengthUnit:
    Px, Percent, CM, MM, In = "Px", "Percent", "CM", "MM", "In"


class Color:
    """java.awt.Color constants as CSS hex strings (the reference serialises colours as hex)."""
    BLACK, WHITE, GRAY, LIGHT_GRAY, DARK_GRAY = "#000000", "#FFFFFF", "#808080", "#C0C0C0", "#404040"
    RED, GREEN, BLUE, YELLOW, CYAN = "#FF0000", "#00FF00", "#0000FF", "#FFFF00", "#00FFFF"
    MAGENTA, ORANGE, PINK = "#FF00FF", "#FFC800", "#FFAFAF"


def _jsonable(v):
    if isinstance(v, Style):
        return v.to_dict()
    if isinstance(v, (list, tuple)):
        return [_jsonable(x) for x in v]
    if hasattr(v, "name") and not isinstance(v, (str, int, float)):
        return v.name
    return v


class Style:
    """Component style: a flat field map (width / height with their units, margins, colours, fonts, ...), built
    with the reference's style builders (StyleChart.Builder().width(640, LengthUnit.Px)...) and serialised as JSON
    with its style type, so fromJson rebuilds an equal style."""
    TYPE = "Style"
    _REGISTRY = {}

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        Style._REGISTRY[cls.TYPE] = cls

    def __init__(self, width=600, height=300, **kw):
        self.width, self.height = width, height
        self.extra = kw

    def to_dict(self):
        return {"styleType": self.TYPE, "width": self.width, "height": self.height, **self.extra}

    def toJson(self):
        return json.dumps(self.to_dict(), sort_keys=True)

    @staticmethod
    def from_dict(d):
        d = dict(d)
        cls = Style._REGISTRY.get(d.pop("styleType", "Style"), Style)
        return cls(**d)

    @staticmethod
    def fromJson(s):
        return Style.from_dict(json.loads(s))

    def __str__(self):
        return f"{self.TYPE}({self.toJson()})"

    def __eq__(self, other):
        return isinstance(other, Style) and self.to_dict() == other.to_dict()

    __hash__ = None

    class _Builder:
        def __init__(self, cls):
            self._cls, self._f = cls, {}

        def __getattr__(self, name):
            if name.startswith("_"):
                raise AttributeError(name)

            def setter(*args):
                if name in ("width", "height") and len(args) == 2:
                    self._f[name], self._f[name + "Unit"] = args[0], _jsonable(args[1])
                else:
                    self._f[name] = _jsonable(args[0] if len(args) == 1 else list(args))
                return self
            return setter

        def build(self):
            f = dict(self._f)
            return self._cls(width=f.pop("width", 600), height=f.pop("height", 300), **f)

    @classmethod
    def Builder(cls):
        return Style._Builder(cls)


class StyleChart(Style):
    TYPE = "StyleChart"


class StyleTable(Style):
    TYPE = "StyleTable"


class StyleText(Style):
    TYPE = "StyleText"


class StyleAccordion(Style):
    TYPE = "StyleAccordion"


class StyleDiv(Style):
    TYPE = "StyleDiv"

    class FloatValue:
        non, left, right, initial, inherit = "non", "left", "right", "initial", "inherit"


_COLORS = ["#1f77b4", "#ff7f0e", "#2ca02c", "#d62728", "#9467bd", "#8c564b", "#e377c2", "#7f7f7f"]


class Component:
    """Base component: JSON round trip through ``toJson`` / ``Component.fromJson`` (the componentType names the
    class, as the reference's Jackson subtypes); ``str()`` is the canonical JSON, so equal components print equal."""
    TYPE = "Component"
    _REGISTRY = {}

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        Component._REGISTRY[cls.TYPE] = cls

    def __init__(self, title=None, style=None):
        self.title = title
        self.style = style or Style()

    def to_dict(self):
        return {"componentType": self.TYPE, "title": self.title, "style": self.style.to_dict()}

    def toJson(self):
        return json.dumps(self.to_dict())

    def _load(self, d):
        """Fill the subclass fields from a to_dict() map (title / style already set)."""

    @staticmethod
    def from_dict(d):
        cls = Component._REGISTRY.get(d.get("componentType"))
        if cls is None:
            raise ValueError(f"unknown component type {d.get('componentType')!r}")
        c = cls.__new__(cls)
        Component.__init__(c, d.get("title"), Style.from_dict(d["style"]) if d.get("style") else None)
        c._load(d)
        return c

    @staticmethod
    def fromJson(s):
        return Component.from_dict(json.loads(s))

    def __str__(self):
        return f"{self.TYPE}({json.dumps(self.to_dict(), sort_keys=True)})"

    def __eq__(self, other):
        return isinstance(other, Component) and self.to_dict() == other.to_dict()

    __hash__ = None

    def render(self):
        raise NotImplementedError

    def _frame(self, body):
        t = f"<h4>{html.escape(self.title)}</h4>" if self.title else ""
        return f'<div class="dl4j-component">{t}{body}</div>'


class _Chart(Component):
    TYPE = "_Chart"
    def __init__(self, title=None, style=None):
        super().__init__(title, style)
        self.series = []            # (name, xs, ys)
        self.options = {}           # gridWidth / showLegend / axis limits (ChartLine / ChartScatter builders)

    def addSeries(self, name, x, y):
        self.series.append((name, [float(v) for v in x], [float(v) for v in y]))
        return self

    def to_dict(self):
        d = super().to_dict()
        d["series"] = [{"name": n, "x": x, "y": y} for n, x, y in self.series]
        if self.options:
            d["options"] = dict(self.options)
        return d

    def _load(self, d):
        self.series = [(e["name"], list(e["x"]), list(e["y"])) for e in d.get("series", [])]
        self.options = dict(d.get("options", {}))

    class _ChartBuilder:
        def __init__(self, cls, title, style):
            self.c = cls(title, style)

        def addSeries(self, name, x, y=None):
            self.c.addSeries(name, x, y) if y is not None else self.c.addSeries(name, x)
            return self

        def setGridWidth(self, x, y):
            self.c.options["gridWidth"] = [x, y]
            return self

        def showLegend(self, b):
            self.c.options["showLegend"] = bool(b)
            return self

        def setXMin(self, v):
            self.c.options["xMin"] = v
            return self

        def setXMax(self, v):
            self.c.options["xMax"] = v
            return self

        def setYMin(self, v):
            self.c.options["yMin"] = v
            return self

        def setYMax(self, v):
            self.c.options["yMax"] = v
            return self

        def setXValues(self, xs):                # ChartStackedArea
            self.c.x = [float(v) for v in xs]
            return self

        def build(self):
            return self.c

    @classmethod
    def Builder(cls, title, style=None):
        return _Chart._ChartBuilder(cls, title, style)

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

    def addSeries(self, name, x, y=None):
        if y is None:                          # Builder form: addSeries(name, yValues) after setXValues
            x, y = getattr(self, "x", list(range(len(x)))), x
        return super().addSeries(name, x, y)

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

    def _load(self, d):
        self.bins = [(e["lower"], e["upper"], e["y"]) for e in d.get("bins", [])]

    class _HB:
        def __init__(self, title, style):
            self.c = ChartHistogram(title, style)

        def addBin(self, lower, upper, y):
            self.c.addBin(lower, upper, y)
            return self

        def build(self):
            return self.c

    @staticmethod
    def Builder(title, style=None):
        return ChartHistogram._HB(title, style)

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

    def _load(self, d):
        self.labels, self.values = list(d.get("labels", [])), list(d.get("values", []))

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

    class TimelineEntry:
        def __init__(self, entryLabel, startTimeMs, endTimeMs, color=None):
            self.entryLabel, self.startTimeMs, self.endTimeMs, self.color = entryLabel, startTimeMs, endTimeMs, color

    def addLaneData(self, name, entries):
        self.lanes.append((name, [(float(a), float(b), str(l)) for a, b, l in entries]))
        return self

    def addLane(self, name, entries):
        """Reference form: a list of TimelineEntry(label, startMs, endMs[, color])."""
        self.lanes.append((name, [(float(e.startTimeMs), float(e.endTimeMs), str(e.entryLabel)) +
                                  ((e.color,) if e.color is not None else ()) for e in entries]))
        return self

    def to_dict(self):
        d = super().to_dict()
        d["lanes"] = [{"name": n, "entries": [list(x) for x in e]} for n, e in self.lanes]
        return d

    def _load(self, d):
        self.lanes = [(e["name"], [tuple(x) for x in e["entries"]]) for e in d.get("lanes", [])]

    class _TB:
        def __init__(self, title, style):
            self.c = ChartTimeline(title, style)

        def addLane(self, name, entries):
            self.c.addLane(name, entries)
            return self

        def build(self):
            return self.c

    @staticmethod
    def Builder(title, style=None):
        return ChartTimeline._TB(title, style)

    def render(self):
        w = self.style.width
        all_t = [t for _, es in self.lanes for a, b, *_ in es for t in (a, b)] or [0, 1]
        t0, t1 = min(all_t), max(all_t)
        span = (t1 - t0) or 1.0
        lh = 20
        out = []
        for i, (n, es) in enumerate(self.lanes):
            out.append(f'<text x="0" y="{i * lh + 14}" font-size="10">{html.escape(n)}</text>')
            for k, (a, b, l, *col) in enumerate(es):
                fill = html.escape(col[0]) if col else _COLORS[k % 8]
                out.append(f'<rect x="{100 + (a - t0) / span * (w - 110):.1f}" y="{i * lh + 3}" '
                           f'width="{max(1.0, (b - a) / span * (w - 110)):.1f}" height="{lh - 6}" '
                           f'fill="{fill}"><title>{html.escape(l)}</title></rect>')
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

    def _load(self, d):
        self.header, self.content = list(d.get("header", [])), [list(r) for r in d.get("content", [])]

    class _TB:
        def __init__(self, style):
            self.c = ComponentTable(style=style)

        def header(self, *h):
            self.c.header = list(h)
            return self

        def content(self, rows):
            self.c.content = [list(r) for r in rows]
            return self

        def build(self):
            return self.c

    @staticmethod
    def Builder(style=None):
        return ComponentTable._TB(style)

    def render(self):
        h = "".join(f"<th>{html.escape(str(c))}</th>" for c in self.header)
        rows = "".join("<tr>" + "".join(f"<td>{html.escape(str(c))}</td>" for c in r) + "</tr>" for r in self.content)
        return self._frame(f'<table border="1" cellpadding="3"><tr>{h}</tr>{rows}</table>')


class ComponentText(Component):
    TYPE = "ComponentText"

    def __init__(self, text="", title=None, style=None):
        if isinstance(title, Style):
            title, style = None, title                   # reference form ComponentText(text, style)
        super().__init__(title, style)
        self.text = text

    def to_dict(self):
        d = super().to_dict()
        d["text"] = self.text
        return d

    def _load(self, d):
        self.text = d.get("text", "")

    class _TB:
        def __init__(self, text, style):
            self.c = ComponentText(text, style=style)

        def build(self):
            return self.c

    @staticmethod
    def Builder(text, style=None):
        return ComponentText._TB(text, style)

    def render(self):
        return self._frame(f"<p>{html.escape(self.text)}</p>")


class ComponentDiv(Component):
    TYPE = "ComponentDiv"

    def __init__(self, *children, style=None):
        if children and isinstance(children[0], Style):  # reference form ComponentDiv(style, components...)
            style, children = children[0], children[1:]
        super().__init__(None, style)
        self.children = list(children)

    def to_dict(self):
        d = super().to_dict()
        d["components"] = [c.to_dict() for c in self.children]
        return d

    def _load(self, d):
        self.children = [Component.from_dict(c) for c in d.get("components", [])]

    def render(self):
        return "<div>" + "".join(c.render() for c in self.children) + "</div>"


class DecoratorAccordion(ComponentDiv):
    TYPE = "DecoratorAccordion"

    def __init__(self, title, *children, defaultCollapsed=False, style=None):
        super().__init__(*children, style=style)
        self.title = title
        self.collapsed = defaultCollapsed

    def to_dict(self):
        d = super().to_dict()
        d["defaultCollapsed"] = bool(self.collapsed)
        return d

    def _load(self, d):
        super()._load(d)
        self.collapsed = bool(d.get("defaultCollapsed", False))

    class _AB:
        def __init__(self, style):
            self.c = DecoratorAccordion(None, style=style)

        def title(self, t):
            self.c.title = t
            return self

        def setDefaultCollapsed(self, b):
            self.c.collapsed = bool(b)
            return self

        def addComponents(self, *cs):
            self.c.children.extend(cs)
            return self

        def build(self):
            return self.c

    @staticmethod
    def Builder(style=None):
        return DecoratorAccordion._AB(style)

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
