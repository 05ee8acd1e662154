// TEST DOUBLE: see NeuralNetworkLayer.hh (the linear part lives in the layer double)
#pragma once
#include "NeuralNetworkLayer.hh"
