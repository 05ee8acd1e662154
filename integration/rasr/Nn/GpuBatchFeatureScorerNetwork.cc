// GpuBatchFeatureScorerNetwork.cc -- GpuBatchFeatureScorer::initNetwork: BatchFeatureScorer::init
// (src/Nn/BatchFeatureScorer.cc:45-79) with the reference's own network, prior and class-label objects, then the
// network's layers handed to nn_scorer_create (include/rasr_nn.h).  Separate from the protocol because the Nn
// headers pull in Math/Blas.hh -> <cblas.h> (src/Math/Blas.hh:28), which an RASR build has and this image lacks.
#include "GpuBatchFeatureScorer.hh"

#include "ClassLabelWrapper.hh"
#include "LinearAndActivationLayer.hh"
#include "LinearLayer.hh"
#include "NeuralNetwork.hh"
#include "Prior.hh"

#include <memory>
#include <vector>

using namespace Nn;

namespace {

// SigmoidLayer's "gamma" (ActivationLayer.cc:102-104), read from the layer's own configuration
const Core::ParameterFloat paramLayerGamma("gamma", "exponential scaling factor", 1.0);

// the activation a layer type applies after its linear part (or on its own), -1 if not supported
int activationOf(NeuralNetworkLayer<f32>::LayerType t, bool* hasLinear) {
    typedef NeuralNetworkLayer<f32> L;
    *hasLinear = false;
    switch (t) {
        case L::linearAndSigmoidLayer: *hasLinear = true; return NN_ACT_SIGMOID;
        case L::linearAndTanhLayer: *hasLinear = true; return NN_ACT_TANH;
        case L::linearAndRectifiedLayer: *hasLinear = true; return NN_ACT_RELU;
        case L::linearAndEluLayer: *hasLinear = true; return NN_ACT_ELU;
        case L::linearAndSoftmaxLayer: *hasLinear = true; return NN_ACT_IDENTITY;  // softmax not evaluated
        case L::linearLayer: *hasLinear = true; return NN_ACT_IDENTITY;
        case L::sigmoidLayer: return NN_ACT_SIGMOID;
        case L::tanhLayer: return NN_ACT_TANH;
        case L::rectifiedLayer: return NN_ACT_RELU;
        case L::eluLayer: return NN_ACT_ELU;
        case L::identityLayer: return NN_ACT_IDENTITY;
        default: return -1;
    }
}

}  // namespace

void GpuBatchFeatureScorer::initNetwork(Core::Ref<const Mm::MixtureSet> mixtureSet) {
    log("initialize gpu-nn-batch-feature-scorer with buffer size ") << bufferSize_;
    nClasses_ = mixtureSet->nMixtures();

    // (a) class label wrapper
    ClassLabelWrapper labels(select("class-labels"), nClasses_);
    if (!labels.isOneToOneMapping())
        error("no one-to-one correspondence between network outputs and classes!");

    // (b) the reference's network object, configured and loaded as the reference's scorer does
    std::unique_ptr<NeuralNetwork<f32>> network(new NeuralNetwork<f32>(getConfiguration()));
    network->initializeNetwork(bufferSize_);
    require_eq(network->getTopLayer().getOutputDimension(), labels.nClassesToAccumulate());
    LinearAndSoftmaxLayer<f32>* topLayer = dynamic_cast<LinearAndSoftmaxLayer<f32>*>(&network->getTopLayer());
    if (!topLayer)
        error("output layer must be of type 'linear+softmax'");
    if (network->getLayer(0).nInputActivations() != 1)
        Core::Component::criticalError("Multiple input streams not implemented in BatchFeatureScorer.");
    inputDimension_ = network->getLayer(0).getInputDimension(0);
    nOutputs_       = network->getTopLayer().getOutputDimension();
    outputIndex_.assign(nClasses_, -1);
    for (u32 e = 0; e < nClasses_; ++e)
        if (labels.isClassToAccumulate(e))
            outputIndex_[e] = static_cast<s32>(labels.getOutputIndexFromClassIndex(e));

    // (c) prior removed from the top layer's bias by the reference's own code (f32, as there)
    Prior<f32> prior(getConfiguration());
    if (prior.fileName() != "")
        prior.read();
    else
        prior.setFromMixtureSet(mixtureSet, labels);
    network->finishComputation();
    topLayer->removeLogPriorFromBias(prior);

    // (d) the chain of layers -> nn_layer_desc: weights [input][output] (weights_.at(input, output),
    // LinearLayer.cc:405-419), bias, the activation that follows the linear part
    std::vector<nn_layer_desc>      descs;
    std::vector<std::vector<float>> weights, biases;
    for (u32 l = 0; l < network->nLayers(); ++l) {
        NeuralNetworkLayer<f32>& layer = network->getLayer(l);
        // a single chain: layer l reads the output of layer l-1 (layer 0 the feature stream); output activation
        // index = layer index + number of feature streams (NeuralNetwork.cc:140-142), one stream here
        const u32 expectedInput = l == 0 ? 0 : network->getLayer(l - 1).getOutputActivationIndex();
        if (layer.nInputActivations() != 1 || layer.getInputActivationIndex(0) != expectedInput ||
            layer.getOutputActivationIndex() != l + 1)
            criticalError("GPU nn scorer: layer %u is not part of a single chain of layers", l);
        bool      hasLinear = false;
        const int act       = activationOf(layer.getLayerType(), &hasLinear);
        if (act < 0)
            criticalError("GPU nn scorer: layer %u: layer type not supported", l);
        const float gamma = act == NN_ACT_SIGMOID ? f32(paramLayerGamma(layer.getConfiguration())) : 1.0f;
        if (!hasLinear) {  // an activation layer after a linear one: fused into it
            if (descs.empty() || descs.back().activation != NN_ACT_IDENTITY ||
                layer.getOutputDimension() != descs.back().output_dim)
                criticalError("GPU nn scorer: layer %u: an activation layer must follow a linear layer", l);
            descs.back().activation = static_cast<nn_activation>(act);
            descs.back().gamma      = gamma;
            continue;
        }
        const NeuralNetworkLayer<f32>::NnMatrix* W = layer.getWeights(0);
        const NeuralNetworkLayer<f32>::NnVector* b = layer.getBias();
        if (!W)
            criticalError("GPU nn scorer: layer %u has no weights", l);
        const u32 nIn = W->nRows(), nOut = W->nColumns();
        weights.push_back(std::vector<float>(static_cast<size_t>(nIn) * nOut));
        for (u32 i = 0; i < nIn; ++i)
            for (u32 o = 0; o < nOut; ++o)
                weights.back()[static_cast<size_t>(i) * nOut + o] = W->at(i, o);
        biases.push_back(std::vector<float>());
        if (b)
            for (u32 o = 0; o < nOut; ++o)
                biases.back().push_back(b->at(o));
        nn_layer_desc d;
        d.input_dim  = nIn;
        d.output_dim = nOut;
        d.weights    = 0;  // set below, once the vectors have stopped moving
        d.bias       = 0;
        d.activation = static_cast<nn_activation>(act);
        d.gamma      = gamma;
        descs.push_back(d);
    }
    if (descs.empty())
        criticalError("GPU nn scorer: empty network");
    for (size_t i = 0; i < descs.size(); ++i) {
        descs[i].weights = &weights[i][0];
        descs[i].bias    = biases[i].empty() ? 0 : &biases[i][0];
    }
    descs.back().activation = NN_ACT_IDENTITY;  // top layer: softmax off (BatchFeatureScorer.cc:58-59)
    nn_network_desc net;
    net.n_layers    = static_cast<uint32_t>(descs.size());
    net.layers      = &descs[0];
    net.log_prior   = 0;  // removed from the bias above, in the reference's arithmetic
    net.prior_scale = 0.0f;
    const int device = paramDevice(getConfiguration());
    if (nn_scorer_create(&net, bufferSize_, device, &scorer_) != GMM_OK)
        criticalError("GPU nn scorer: %s", nn_last_error());
    log("gpu-nn-batch-feature-scorer: ") << descs.size() << " layers on device " << device << ", buffer size "
                                         << bufferSize_;
}
