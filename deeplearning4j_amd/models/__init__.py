"""Model zoo (reference deeplearning4j-zoo)."""
from .labels import (BaseLabels, ClassPrediction, COCOLabels, DarknetLabels, ImageNetLabels, VOCLabels,  # noqa
                     adler32_file)
from .zoo import (ZOO, AlexNet, BertBase, Darknet19, FaceNetNN4Small2, GoogLeNet, InceptionResNetV1, LeNet, ResNet50,  # noqa
                  ModelMetaData, ModelSelector, PretrainedType, SimpleCNN, TextGenerationLSTM, TinyYOLO, VGG16, VGG19,
                  YOLO2, ZooModel, ZooType)
