"""Runtime layer implementations (one module per family)."""
