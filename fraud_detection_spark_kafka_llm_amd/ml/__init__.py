"""Spark-ML-compatible API (pyspark.ml surface used by the reference)."""
from .base import Estimator, Model, Param, Params, Pipeline, PipelineModel, Transformer
from .classification import (DecisionTreeClassificationModel, DecisionTreeClassifier, LogisticRegression,
                             LogisticRegressionModel, RandomForestClassificationModel, RandomForestClassifier)
from .feature import IDF, CountVectorizer, CountVectorizerModel, HashingTF, IDFModel, StopWordsRemover, Tokenizer
from .frame import Frame, Row, TextColumn, TokenColumn
from .fused import FusedPipeline
from .linalg import DenseVector, SparseVector, VectorColumn, Vectors
