"""Datasets: containers, iterators, fetchers (reference deeplearning4j-data)."""
from .dataset import (DataSet, DataSetIterator, ExistingDataSetIterator, IteratorDataSetIterator,
                      ListDataSetIterator, MultiDataSet, MultiDataSetIterator, SplitTestAndTrain)
from .iterators import (AsyncDataSetIterator, AsyncMultiDataSetIterator, BenchmarkDataSetIterator,
                        BenchmarkMultiDataSetIterator, DoublesDataSetIterator, EarlyTerminationDataSetIterator,
                        KFoldIterator, MultipleEpochsIterator, SamplingDataSetIterator)
