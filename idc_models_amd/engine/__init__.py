from . import losses, metrics, optimizers
from .arena import ParamArena
from .callbacks import Callback, History, JSONLLogger, ModelCheckpoint
from .model import EagerStep, Model, current_strategy, strategy_scope
from .optimizers import SGD, RMSprop

__all__ = ["losses", "metrics", "optimizers", "ParamArena", "Callback", "History", "JSONLLogger",
           "ModelCheckpoint", "EagerStep", "Model", "current_strategy", "strategy_scope", "SGD",
           "RMSprop"]
