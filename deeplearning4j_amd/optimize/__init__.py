"""Training drivers: listeners, solvers/optimizers, step functions, termination conditions, gradient accumulation
(reference deeplearning4j-nn/src/main/java/org/deeplearning4j/optimize/**)."""
from .listeners import (BaseTrainingListener, Checkpoint, CheckpointListener, CollectScoresIterationListener,
                        ComposableIterationListener, EvaluativeListener, InvocationType, IterationListener,
                        ParamAndGradientIterationListener, PerformanceListener, ScoreIterationListener,
                        SleepyTrainingListener, TimeIterationListener, TrainingListener)
from .solvers import (LBFGS, BackTrackLineSearch, ConjugateGradient, DefaultStepFunction, EpsTermination,
                      GradientStepFunction, LineGradientDescent, NegativeDefaultStepFunction,
                      NegativeGradientStepFunction, Norm2Termination, Solver, StochasticGradientDescent,
                      ZeroDirection)
