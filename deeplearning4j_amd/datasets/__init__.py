"""Datasets: containers, iterators, fetchers (reference deeplearning4j-data)."""
from .dataset import (DataSet, DataSetIterator, ExistingDataSetIterator, IteratorDataSetIterator,
                      ListDataSetIterator, MultiDataSet, MultiDataSetIterator, SplitTestAndTrain)
from .iterators import (AsyncDataSetIterator, AsyncMultiDataSetIterator, BenchmarkDataSetIterator,
                        BenchmarkMultiDataSetIterator, DoublesDataSetIterator, EarlyTerminationDataSetIterator,
                        KFoldIterator, MultiDataSetIteratorAdapter, MultipleEpochsIterator, SamplingDataSetIterator, DataSetIteratorSplitter,
                        FileDataSetIterator, ReconstructionDataSetIterator, InequalityHandling,
                        JointParallelDataSetIterator, CombinedPreProcessor, CombinedMultiDataSetPreProcessor,
                        BaseParallelDataSetIterator, FileSplitDataSetIterator, FileSplitParallelDataSetIterator,
                        EarlyTerminationMultiDataSetIterator, FloatsDataSetIterator, INDArrayDataSetIterator,
                        MultiDataSetIteratorSplitter)
from .normalizers import (NormalizerStandardize, NormalizerMinMaxScaler, ImagePreProcessingScaler,  # noqa: F401
                          VGG16ImagePreProcessor, MultiNormalizerStandardize, MultiNormalizerMinMaxScaler)
from .fetchers import (CifarDataSetIterator, EmnistDataSetIterator, IrisDataSetIterator, LFWDataSetIterator,  # noqa
                       MnistDataSetIterator, TinyImageNetDataSetIterator, UciSequenceDataSetIterator)
from .datavec import (CSVRecordReader, CSVSequenceRecordReader, CollectionRecordReader, FileSplit,  # noqa: F401
                      ImageRecordReader, RecordReaderDataSetIterator, RecordReaderMultiDataSetIterator,
                      SequenceRecordReaderDataSetIterator)
