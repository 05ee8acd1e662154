// TEST DOUBLE: Mm index / score types (src/Mm/Types.hh names)
#pragma once
#include <string>
#include <vector>
#include <Core/Types.hh>
namespace Mm {
typedef f32                      Score;
typedef f32                      FeatureType;
typedef f32                      MeanType;
typedef f32                      VarianceType;
typedef f64                      Weight;
typedef u32                      ComponentIndex;
typedef u32                      MixtureIndex;
typedef MixtureIndex             EmissionIndex;
typedef u32                      DensityIndex;
typedef u32                      DensityInMixture;
typedef u32                      MeanIndex;
typedef u32                      CovarianceIndex;
typedef std::vector<FeatureType> FeatureVector;
}  // namespace Mm
