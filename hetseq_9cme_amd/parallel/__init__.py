from . import distributed  # noqa: F401
from .flat_params import FlatParamSpace  # noqa: F401
from .reducer import GradReducer  # noqa: F401
