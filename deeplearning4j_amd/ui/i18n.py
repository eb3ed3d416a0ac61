"""Internationalisation of the training UI (reference PLAY:i18n/I18NProvider.java, DefaultI18N.java: per-language
message maps keyed like ``train.nav.overview``, a session-wide current language switched by ``/setlang/:to``, falling
back to English for a key a language lacks).

Messages are defined here, not loaded from the reference's resource files. Languages: en, de, ja, ko, ru, zh.
"""
import threading

DEFAULT_LANGUAGE = "en"

_MESSAGES = {
    "en": {
        "train.pagetitle": "DL4J-AMD Training UI",
        "train.nav.overview": "Overview", "train.nav.model": "Model", "train.nav.system": "System",
        "train.nav.help": "Help", "train.nav.language": "Language", "train.nav.session": "Session",
        "train.nav.worker": "Worker",
        "train.overview.title": "Training overview",
        "train.overview.chart.scoreTitle": "Score vs. iteration",
        "train.overview.chart.updateRatioTitle": "Update : parameter ratio (log10 mean magnitude)",
        "train.overview.chart.perfTitle": "Examples / second",
        "train.overview.perftable.startTime": "Model start time",
        "train.overview.perftable.totalRuntime": "Total runtime",
        "train.overview.perftable.lastUpdate": "Last update",
        "train.overview.perftable.totalParamUpdates": "Total parameter updates",
        "train.overview.perftable.updatesPerSec": "Updates / second",
        "train.overview.perftable.examplesPerSec": "Examples / second",
        "train.overview.modeltable.modeltype": "Model type",
        "train.overview.modeltable.nLayers": "Number of layers",
        "train.overview.modeltable.nParams": "Number of parameters",
        "train.model.title": "Model", "train.model.layerInfoTable.title": "Layer information",
        "train.model.meanmag.title": "Mean magnitudes (parameters and updates)",
        "train.model.lrChart.title": "Learning rate",
        "train.model.paramHistChart.title": "Parameter histogram",
        "train.model.updateHistChart.title": "Update histogram",
        "train.system.title": "System", "train.system.hwTable.title": "Hardware",
        "train.system.swTable.title": "Software", "train.system.chart.memory": "Memory utilisation",
        "train.help.title": "Help",
        "train.help.text": "Attach a StatsStorage to the UIServer and add a StatsListener to the network.",
        "train.session.none": "No sessions", "activations.title": "Convolutional activations",
        "tsne.title": "t-SNE", "tsne.upload": "Upload coordinates (x,y,label per line)",
    },
    "de": {
        "train.nav.overview": "Übersicht", "train.nav.model": "Modell", "train.nav.system": "System",
        "train.nav.help": "Hilfe", "train.nav.language": "Sprache", "train.nav.session": "Sitzung",
        "train.overview.title": "Trainingsübersicht",
        "train.overview.chart.scoreTitle": "Score pro Iteration",
        "train.overview.chart.perfTitle": "Beispiele / Sekunde",
        "train.overview.modeltable.nLayers": "Anzahl der Schichten",
        "train.overview.modeltable.nParams": "Anzahl der Parameter",
        "train.model.title": "Modell", "train.system.title": "System", "train.help.title": "Hilfe",
    },
    "ja": {
        "train.nav.overview": "概要", "train.nav.model": "モデル", "train.nav.system": "システム",
        "train.nav.help": "ヘルプ", "train.nav.language": "言語", "train.nav.session": "セッション",
        "train.overview.title": "学習の概要", "train.overview.chart.scoreTitle": "スコアと反復回数",
        "train.overview.chart.perfTitle": "サンプル数 / 秒", "train.model.title": "モデル",
        "train.system.title": "システム", "train.help.title": "ヘルプ",
    },
    "ko": {
        "train.nav.overview": "개요", "train.nav.model": "모델", "train.nav.system": "시스템",
        "train.nav.help": "도움말", "train.nav.language": "언어", "train.nav.session": "세션",
        "train.overview.title": "학습 개요", "train.overview.chart.scoreTitle": "반복별 점수",
        "train.model.title": "모델", "train.system.title": "시스템", "train.help.title": "도움말",
    },
    "ru": {
        "train.nav.overview": "Обзор", "train.nav.model": "Модель", "train.nav.system": "Система",
        "train.nav.help": "Справка", "train.nav.language": "Язык", "train.nav.session": "Сеанс",
        "train.overview.title": "Обзор обучения", "train.overview.chart.scoreTitle": "Оценка по итерациям",
        "train.model.title": "Модель", "train.system.title": "Система", "train.help.title": "Справка",
    },
    "zh": {
        "train.nav.overview": "概览", "train.nav.model": "模型", "train.nav.system": "系统",
        "train.nav.help": "帮助", "train.nav.language": "语言", "train.nav.session": "会话",
        "train.overview.title": "训练概览", "train.overview.chart.scoreTitle": "得分与迭代次数",
        "train.model.title": "模型", "train.system.title": "系统", "train.help.title": "帮助",
    },
}


class DefaultI18N:
    """Message lookup with an English fallback; ``setDefaultLanguage`` is what ``/setlang/:to`` calls."""
    _instance = None
    _lock = threading.Lock()

    def __init__(self):
        self.current = DEFAULT_LANGUAGE

    @staticmethod
    def getInstance():
        with DefaultI18N._lock:
            if DefaultI18N._instance is None:
                DefaultI18N._instance = DefaultI18N()
            return DefaultI18N._instance

    def getMessage(self, key, langCode=None):
        lang = langCode or self.current
        m = _MESSAGES.get(lang, {})
        return m.get(key, _MESSAGES[DEFAULT_LANGUAGE].get(key, key))

    def getDefaultLanguage(self):
        return self.current

    def setDefaultLanguage(self, lang):
        if lang not in _MESSAGES:
            raise ValueError(f"unsupported UI language {lang!r}; have {sorted(_MESSAGES)}")
        self.current = lang

    @staticmethod
    def languages():
        return sorted(_MESSAGES)

    def messages(self, langCode=None):
        """Every key of the current (or given) language, English filling the gaps."""
        out = dict(_MESSAGES[DEFAULT_LANGUAGE])
        out.update(_MESSAGES.get(langCode or self.current, {}))
        return out


class I18NProvider:
    @staticmethod
    def getInstance():
        return DefaultI18N.getInstance()
