"""NLP: tokenization, vocabularies and embedding learners (Word2Vec, ParagraphVectors, GloVe) on the native
batcher + gfx950 embedding kernels; WordVectorSerializer formats."""
from .text import *  # noqa: F401,F403
from .vocab import AbstractCache, Huffman, InMemoryLookupCache, SequenceElement, VocabConstructor, VocabWord  # noqa
from .embeddings import EmbeddingEngine, InMemoryLookupTable, WordVectorsImpl  # noqa: F401
from .word2vec import (CBOW, DBOW, DM, ParagraphVectors, ScoreListener, SequenceVectors, SerializingListener,  # noqa
                       SkipGram, VectorsConfiguration, VectorsListener, Word2Vec)
from .tokenization_ext import (BertWordPieceTokenizerFactory, ChineseTokenizerFactory,  # noqa: F401
                               JapaneseTokenizerFactory, KoreanTokenizerFactory, PorterStemmer, StemmingPreprocessor)
from .distributed import DistributedWord2Vec, SparkWord2Vec  # noqa: F401
from .text import ContextLabelRetriever  # noqa: F401,E402
