"""Model zoo (reference deeplearning4j-zoo)."""
from .zoo import (ZOO, AlexNet, Darknet19, GoogLeNet, LeNet, ResNet50, SimpleCNN, TextGenerationLSTM, VGG16, VGG19,
                  ZooModel)
