"""paddle.vision: model zoo, synthetic datasets and basic transforms."""
from . import datasets, models, transforms  # noqa: F401
from .models import LeNet, ResNet, resnet18, resnet34, resnet50, resnet101, resnet152, vgg16  # noqa: F401
