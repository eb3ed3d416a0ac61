"""Model zoo (reference deeplearning4j-zoo)."""
from .zoo import (ZOO, AlexNet, BertBase, Darknet19, FaceNetNN4Small2, GoogLeNet, InceptionResNetV1, LeNet, ResNet50,  # noqa
                  SimpleCNN, TextGenerationLSTM, TinyYOLO, VGG16, VGG19, YOLO2, ZooModel)
