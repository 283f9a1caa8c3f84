/* TEST-ONLY stand-in for ORB_SLAM2/include/ORBVocabulary.h (the DBoW2 TemplatedVocabulary typedef):
 * the drop-ins only use the pointer as the key of their device-vocabulary registry. */
#ifndef ORBVOCABULARY_H
#define ORBVOCABULARY_H
namespace ORB_SLAM2 {
class ORBVocabulary {};
}  // namespace ORB_SLAM2
#endif
