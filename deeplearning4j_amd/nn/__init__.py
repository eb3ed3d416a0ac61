"""Model layer: configs, runtime layers, MultiLayerNetwork, ComputationGraph, updaters."""
