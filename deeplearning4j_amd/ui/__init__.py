"""Observability: stats listener (fused HIP segment statistics), storage (in-memory / SQLite / remote router),
UI server, static HTML components and the convolutional activations listener."""
from .storage import (CollectionStatsStorageRouter, FileStatsStorage, InMemoryStatsStorage, J7FileStatsStorage,  # noqa
                      Persistable, RemoteUIStatsStorageRouter, StatsStorageEvent, StatsStorageListener,
                      StatsStorageRouter, StorageMetaData)
from .stats import (StatsInitializationConfiguration, StatsListener, StatsType, StatsUpdateConfiguration,  # noqa
                    SummaryType, summarize)
from .server import UIServer  # noqa: F401
from .histogram import HistogramBin  # noqa: F401
from .storage import SbeStorageMetaData, StorageMetaData  # noqa: F401
from .connection import UiConnectionInfo  # noqa: F401,E402
