from .computation_graph import ComputationGraph
